"""Per-op timing of the conv GEMMs at the step's 1024x512 shapes (GPU), for same-box A/B of kernel forms.

    python scripts/bench_ops.py [--reps N] [--check] [--only NAME] [--nimg 2]

Each op call (the C-ABI entry point as ops.py issues it, incl. its reduce and split launches) is timed
with HIP events over `reps` back-to-back calls after warm-up, on f16x3 (the default fp32 form).  Two
builds compare on one box by running this once per library (MSL_LIB_PATH, scripts/gpu_ab.sh).
--check also compares the outputs against fp64 (per-element error relative to the sum of |terms|).
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from maxsquareloss_amd import hip, ops  # noqa: E402

DEV = "cuda"
H, W = 65, 129


def timed(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3  # us


def conv_ops(name, cin, cout, k, d, nb=1, h=H, w=W, nimg=1, dgrad_mode="plain"):
    """(label, fwd, dgrad, wgrad callables, flops, reference checker) for one conv shape."""
    g = torch.Generator().manual_seed(cin + cout)
    x = torch.relu(torch.randn(1, cin, nimg, h, w, generator=g)).to(DEV)  # [C][nimg][h][w]
    wt = (torch.randn(cout, cin, k, k, generator=g) * 0.02).to(DEV)
    gy = torch.randn(1, cout, nimg, h, w, generator=g).to(DEV)
    lib = hip.load()
    s = hip.stream_ptr()
    p = h * w * nimg
    cnt = hip.forms()
    cache = ops.PackCache(pointwise=(k == 1))
    xpart = ops._parts(x)
    gpart = ops._parts(gy)
    y = torch.empty(1, cout, nimg, h, w, device=DEV)
    dx = torch.empty(1, cin, nimg, h, w, device=DEV)
    dw = torch.empty_like(wt)
    if k == 1:
        pf, pd = cache.get([wt], cin, cout, 0), cache.get([wt], cin, cout, 1)
        wsf = hip.workspace(lib.msl_pconv_fwd_workspace(cin, cout, p), DEV)
        wsd = hip.workspace(lib.msl_pconv_dgrad_workspace(cin, cout, p), DEV)
        wsw = hip.workspace(lib.msl_pconv_wgrad_workspace(cin, cout, p), DEV)
        fwd = lambda: hip.check(lib.msl_pconv_fwd_sc(x.data_ptr(), pf.data_ptr(), y.data_ptr(), cin, cout, p, cnt,  # noqa: E731
                                                     wsf.data_ptr(), wsf.numel(), s, *ops._pp(xpart)), "fwd")
        dgr = lambda: hip.check(lib.msl_pconv_dgrad_acc_sc(gy.data_ptr(), pd.data_ptr(), dx.data_ptr(), cin, cout, p,  # noqa: E731
                                                           int(dgrad_mode == "acc"), cnt, wsd.data_ptr(), wsd.numel(), s,
                                                           *ops._pp(gpart)), "dgrad")
        if dgrad_mode == "resmask":  # r06: the masked residual gradient added in the epilogue (timing only)
            res = torch.randn(1, cin, nimg, h, w, generator=g).to(DEV)
            bits = torch.randint(-2**62, 2**62, (cin * nimg * ((h * w + 63) // 64),), generator=g).to(DEV)
            dgr = lambda: hip.check(lib.msl_pconv_dgrad_resmask_sc(  # noqa: E731
                gy.data_ptr(), pd.data_ptr(), dx.data_ptr(), cin, cout, p, res.data_ptr(), bits.data_ptr(), nimg, cnt,
                wsd.data_ptr(), wsd.numel(), s, *ops._pp(gpart)), "dgrad")
        wgr = lambda: hip.check(lib.msl_pconv_wgrad_sc(x.data_ptr(), gy.data_ptr(), dw.data_ptr(), cin, cout, p, 0,  # noqa: E731
                                                       cnt, wsw.data_ptr(), wsw.numel(), s, *ops._pp(xpart),
                                                       *ops._pp(gpart)), "wgrad")
        ref = lambda xx, ww: F.conv2d(xx, ww)  # noqa: E731
    else:
        pf, pd = cache.get([wt], cin, cout, 0), cache.get([wt], cin, cout, 1)
        wsf = hip.workspace(lib.msl_dconv_fwd_workspace(1, cin, cout, h, w, nimg), DEV)
        wsd = hip.workspace(lib.msl_dconv_dgrad_workspace(1, cin, cout, h, w, nimg), DEV)
        wsw = hip.workspace(lib.msl_dconv_wgrad_workspace(1, cin, cout, h, w, nimg), DEV)
        fwd = lambda: hip.check(lib.msl_dconv_fwd_sc(x.data_ptr(), pf.data_ptr(), None, y.data_ptr(), 1, cin, cout,  # noqa: E731
                                                     h, w, nimg, d, 0, cnt, wsf.data_ptr(), wsf.numel(), s,
                                                     *ops._pp(xpart)), "fwd")
        dgr = lambda: hip.check(lib.msl_dconv_dgrad_sc(gy.data_ptr(), pd.data_ptr(), dx.data_ptr(), 1, cin, cout, h,  # noqa: E731
                                                       w, nimg, d, 0, cnt, wsd.data_ptr(), wsd.numel(), s,
                                                       *ops._pp(gpart)), "dgrad")
        wgr = lambda: hip.check(lib.msl_dconv_wgrad_sc(x.data_ptr(), gy.data_ptr(), dw.data_ptr(), None, 1, cin,  # noqa: E731
                                                       cout, h, w, nimg, d, 0, 0, cnt, wsw.data_ptr(), wsw.numel(), s,
                                                       *ops._pp(xpart), *ops._pp(gpart)), "wgrad")
        ref = lambda xx, ww: F.conv2d(xx, ww, padding=d, dilation=d)  # noqa: E731
    flops = 2.0 * cin * cout * k * k * p  # p counts every image

    def nchw(t):  # [1][C][nimg][h][w] -> the images as an NCHW batch, fp64 on the host
        return t.double().cpu()[0].transpose(0, 1).contiguous()

    def check():
        xr, wr = nchw(x).requires_grad_(), wt.double().cpu().requires_grad_()
        yr = ref(xr, wr)
        yr.backward(nchw(gy))
        xa, wa = nchw(x).abs().requires_grad_(), wt.double().cpu().abs().requires_grad_()
        ya = ref(xa, wa)
        ya.backward(nchw(gy).abs())
        fwd(); dgr(); wgr()  # noqa: E702
        torch.cuda.synchronize()
        e = lambda o, r, b: ((o - r).abs() / b.clamp_min(1e-300)).max().item()  # noqa: E731
        return (e(nchw(y), yr.detach(), ya.detach()), e(nchw(dx), xr.grad, xa.grad),
                e(dw.double().cpu(), wr.grad, wa.grad))
    return name, fwd, dgr, wgr, flops, check


SHAPES = [("aspp6 2048->19", 2048, 19, 3, 6), ("layer1 3x3", 64, 64, 3, 1), ("layer3 3x3 d2", 256, 256, 3, 2), ("layer4 3x3 d4", 512, 512, 3, 4), ("layer2 3x3", 128, 128, 3, 1),
          ("1x1 256->1024", 256, 1024, 1, 0), ("1x1 1024->256", 1024, 256, 1, 0), ("1x1 2048->512", 2048, 512, 1, 0),
          ("1x1 512->2048", 512, 2048, 1, 0), ("1x1 256->64", 256, 64, 1, 0), ("1x1 64->256", 64, 256, 1, 0),
          ("aspp shift 2048->342", 2048, 342, 1, 0)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--only", default=None, help="substring of the shape names to run")
    ap.add_argument("--hw", type=int, nargs=2, default=[H, W], help="map size (default the step's 65 x 129)")
    ap.add_argument("--nimg", type=int, default=1, help="images per call ([C][nimg][h][w]; 2 = the trainer's pair)")
    ap.add_argument("--which", default="fwd,dgrad,wgrad", help="the ops to time (a profiler pass over one of them)")
    ap.add_argument("--form", default=None, help="the fp32 form (mfma_f32, bf16x6, f16x3; default: the library's)")
    ap.add_argument("--dgrad-mode", default="plain", choices=["plain", "acc", "resmask"],
                    help="1x1 data gradient: dx =, dx +=, or dx = masked residual + (msl_pconv_dgrad_resmask)")
    a = ap.parse_args()
    if a.form:
        ops.set_f32_form(a.form)
    which = a.which.split(",")
    lib = hip.load()
    ops_list = [conv_ops(*s, h=a.hw[0], w=a.hw[1], nimg=a.nimg, dgrad_mode=a.dgrad_mode) for s in SHAPES if a.only is None or a.only in s[0]]
    for name, fwd, dgr, wgr, flops, check in ops_list:
        t = [timed(f, a.reps) if n in which else float("nan") for n, f in (("fwd", fwd), ("dgrad", dgr), ("wgrad", wgr))]
        rec = {"hw": a.hw, "nimg": a.nimg, "form": ops.f32_form(), "op": name, "dgrad_mode": a.dgrad_mode, "fwd_us": round(t[0], 1), "dgrad_us": round(t[1], 1),
               "wgrad_us": round(t[2], 1), "fwd_tf": round(flops / t[0] / 1e6, 1),
               "wgrad_tf": round(flops / t[2] / 1e6, 1)}
        if a.check:
            rec["err_fwd_dgrad_wgrad"] = [float(f"{e:.2e}") for e in check()]
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
