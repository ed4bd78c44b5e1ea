"""Same-box A/B of the fp32 conv forms (bf16x6 vs f16x3, exact f32 MFMA for reference) on the
hot GEMM shapes at 1024x512: forward, data gradient and weight gradient per op call, timed with
HIP events over 20 calls after warm-up.  Prints one JSON line per (shape, form)."""
import json
import sys

import torch

sys.path.insert(0, ".")
from maxsquareloss_amd import hip, ops  # noqa: E402


def timeit(fn, iters=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def case(name, cin, cout, h, w, d, forms):
    torch.manual_seed(0)
    x = torch.relu(torch.randn(1, cin, h, w, device="cuda"))
    wt = torch.randn(cout, cin, 3 if d else 1, 3 if d else 1, device="cuda") * 0.01
    gy = torch.randn(1, cout, h, w, device="cuda") * 1e-6
    lib = hip.load()
    st = hip.stream_ptr()
    p = h * w
    flops = 2.0 * cin * cout * (9 if d else 1) * p
    for form in forms:
        ops.set_f32_form(form)
        cache = ops.PackCache(pointwise=not d)
        taps = 9 if d else 1
        pk = cache.get([wt], cin, cout, 0)
        pd = cache.get([wt], cin, cout, 1)
        y = torch.empty(1, cout, h, w, device="cuda")
        dx = torch.empty_like(x)
        dw = torch.empty_like(wt)
        cnt = hip.counters(x.device).data_ptr()
        if d:
            wf = lib.msl_dconv_fwd_workspace(1, cin, cout, h, w, 1)
            wd = lib.msl_dconv_dgrad_workspace(1, cin, cout, h, w, 1)
            ww = lib.msl_dconv_wgrad_workspace(1, cin, cout, h, w, 1)
        else:
            wf = lib.msl_pconv_fwd_workspace(cin, cout, p)
            wd = lib.msl_pconv_dgrad_workspace(cin, cout, p)
            ww = lib.msl_pconv_wgrad_workspace(cin, cout, p)
        wsf = torch.empty(wf, dtype=torch.uint8, device="cuda")
        wsd = torch.empty(wd, dtype=torch.uint8, device="cuda")
        wsw = torch.empty(ww, dtype=torch.uint8, device="cuda")
        if d:
            fwd = lambda: hip.check(lib.msl_dconv_fwd(x.data_ptr(), pk.data_ptr(), None, y.data_ptr(), 1, cin, cout, h, w, 1,
                                                      d, 0, cnt, wsf.data_ptr(), wf, st), "fwd")
            dgr = lambda: hip.check(lib.msl_dconv_dgrad(gy.data_ptr(), pd.data_ptr(), dx.data_ptr(), 1, cin, cout, h, w, 1,
                                                        d, 0, cnt, wsd.data_ptr(), wd, st), "dgrad")
            wgr = lambda: hip.check(lib.msl_dconv_wgrad(x.data_ptr(), gy.data_ptr(), dw.data_ptr(), None, 1, cin, cout,
                                                        h, w, 1, d, 0, 0, wsw.data_ptr(), ww, st), "wgrad")
        else:
            fwd = lambda: hip.check(lib.msl_pconv_fwd(x.data_ptr(), pk.data_ptr(), y.data_ptr(), cin, cout, p, cnt,
                                                      wsf.data_ptr(), wf, st), "fwd")
            dgr = lambda: hip.check(lib.msl_pconv_dgrad(gy.data_ptr(), pd.data_ptr(), dx.data_ptr(), cin, cout, p, cnt,
                                                        wsd.data_ptr(), wd, st), "dgrad")
            wgr = lambda: hip.check(lib.msl_pconv_wgrad(x.data_ptr(), gy.data_ptr(), dw.data_ptr(), cin, cout, p, 0,
                                                        wsw.data_ptr(), ww, st), "wgrad")
        res = {"op": name, "form": form, "shape": [cin, cout, h, w, d]}
        for k, fn in (("fwd_us", fwd), ("dgrad_us", dgr), ("wgrad_us", wgr)):
            res[k] = round(timeit(fn), 2)
        res["fwd_tflops"] = round(flops / res["fwd_us"] / 1e6, 1)
        def repack():
            cache.key[0] = None  # stale: the next get() packs again
            cache.get([wt], cin, cout, 0)
        res["pack_us"] = round(timeit(repack), 2)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    forms = sys.argv[1].split(",") if len(sys.argv) > 1 else ["bf16x6", "f16x3"]
    for rep in range(2):
        case("layer3_d2", 256, 256, 65, 129, 2, forms)
        case("layer4_d4", 512, 512, 65, 129, 4, forms)
        case("pw_1024_256", 1024, 256, 65, 129, 0, forms)
        case("pw_256_1024", 256, 1024, 65, 129, 0, forms)
        case("pw_2048_512", 2048, 512, 65, 129, 0, forms)
