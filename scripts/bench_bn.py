"""Per-call timing of the train-mode BN kernels at the step's pair shapes (GPU), for same-box A/B.

    python scripts/bench_bn.py [--reps N]

For each (channels, residual, relu) of the 1024x512 step's BN layers (p = 65 x 129 per image, two
images per call) times msl_bn_fwd_am and msl_bn_bwd_am_beta (with y, and with y = NULL: the ReLU
mask recomputed from x) with HIP events over `reps` back-to-back calls, and prints one JSON line per
shape with the microseconds and the algorithmic bytes / time.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from maxsquareloss_amd import hip  # noqa: E402

DEV = "cuda"


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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--hw", type=int, nargs=2, default=[65, 129])
    ap.add_argument("--nimg", type=int, default=2)
    ap.add_argument("--unfused", action="store_true", help="the two-kernel form (k_bn_stats + k_bn_apply)")
    args = ap.parse_args()
    lib = hip.load()
    if args.unfused:
        hip.set_form("bn_fused", 0)
    p = args.hw[0] * args.hw[1]
    n = args.nimg
    s = hip.stream_ptr()
    for c, res, relu in [(128, False, True), (256, False, True), (512, False, True), (1024, True, True),
                         (1024, False, False), (2048, True, True), (512, True, True)]:
        g = torch.Generator().manual_seed(c)
        x = (torch.randn(c, n * p, generator=g) * 3 + 1).to(DEV)
        r = torch.randn(c, n * p, generator=g).to(DEV) if res else None
        gamma = (torch.rand(c, generator=g) + 0.5).to(DEV)
        beta = torch.randn(c, generator=g).to(DEV)
        gy = torch.randn(c, n * p, generator=g).to(DEV)
        y, dx, dres = torch.empty_like(x), torch.empty_like(x), torch.empty_like(x) if res else None
        rm, rv = torch.zeros(c, device=DEV), torch.ones(c, device=DEV)
        sm, si = torch.empty(c * n, device=DEV), torch.empty(c * n, device=DEV)
        dg, db, fa, ba = (torch.empty(c, device=DEV) for _ in range(4))
        wsb = lib.msl_bn_workspace(c, p, n)
        ws = hip.workspace(wsb, x.device)

        def fwd():
            hip.check(lib.msl_bn_fwd_am(x.data_ptr(), gamma.data_ptr(), beta.data_ptr(), hip.ptr(r), y.data_ptr(),
                                        rm.data_ptr(), rv.data_ptr(), None, sm.data_ptr(), si.data_ptr(), c, p, n, 1,
                                        1, 0.1, 1e-5, int(relu), hip.forms(), ws.data_ptr(), wsb, s,
                                        fa.data_ptr()), "fwd")

        def bwd(with_y):
            def f():
                hip.check(lib.msl_bn_bwd_am_beta(gy.data_ptr(), x.data_ptr(), y.data_ptr() if with_y else None,
                                                 gamma.data_ptr(), beta.data_ptr(), sm.data_ptr(), si.data_ptr(),
                                                 dx.data_ptr(), hip.ptr(dres), dg.data_ptr(), db.data_ptr(), c, p, n,
                                                 1, int(relu), 0, hip.forms(), ws.data_ptr(), wsb, s,
                                                 ba.data_ptr()), "bwd")
            return f

        mb = c * n * p * 4 / 1e6
        rec = {"c": c, "res": res, "relu": relu, "p": p, "nimg": n, "fused": lib.msl_bn_uses_fused(c, p, 1, hip.forms())}
        t = timed(fwd, args.reps)
        rec["fwd_us"] = round(t, 2)
        rec["fwd_TBps"] = round(mb * (3 if res else 2) / t, 3)
        t = timed(bwd(True), args.reps)
        rec["bwd_us"] = round(t, 2)
        rec["bwd_TBps"] = round(mb * ((3 if relu else 2) + (2 if res else 1)) / t, 3)
        if relu and res and not args.unfused:  # r05: the ReLU mask as bits (msl_bn_fwd_mask / msl_bn_bwd_mask)
            bits = torch.empty(lib.msl_bn_relu_mask_bytes(c, p, n) // 8, dtype=torch.int64, device=DEV)

            def fwdm():
                hip.check(lib.msl_bn_fwd_mask(x.data_ptr(), gamma.data_ptr(), beta.data_ptr(), hip.ptr(r), y.data_ptr(),
                                              rm.data_ptr(), rv.data_ptr(), None, sm.data_ptr(), si.data_ptr(), c, p,
                                              n, 1, 1, 0.1, 1e-5, int(relu), hip.forms(), ws.data_ptr(), wsb, s,
                                              fa.data_ptr(), bits.data_ptr()), "fwd_mask")

            def bwdm():
                hip.check(lib.msl_bn_bwd_mask(gy.data_ptr(), x.data_ptr(), bits.data_ptr(), gamma.data_ptr(),
                                              beta.data_ptr(), sm.data_ptr(), si.data_ptr(), dx.data_ptr(),
                                              hip.ptr(dres), dg.data_ptr(), db.data_ptr(), c, p, n, 1, int(relu), 0,
                                              hip.forms(), ws.data_ptr(), wsb, s, ba.data_ptr()), "bwd_mask")
            def bwdm_nodres():  # r06: the identity block's backward (ops.MaskedResidual: no residual gradient)
                hip.check(lib.msl_bn_bwd_mask(gy.data_ptr(), x.data_ptr(), bits.data_ptr(), gamma.data_ptr(),
                                              beta.data_ptr(), sm.data_ptr(), si.data_ptr(), dx.data_ptr(),
                                              None, dg.data_ptr(), db.data_ptr(), c, p, n, 1, int(relu), 0,
                                              hip.forms(), ws.data_ptr(), wsb, s, ba.data_ptr()), "bwd_mask")
            rec["fwd_mask_us"] = round(timed(fwdm, args.reps), 2)
            rec["fwd_mask_TBps"] = round(mb * 3 / rec["fwd_mask_us"], 3)
            rec["bwd_mask_us"] = round(timed(bwdm, args.reps), 2)
            rec["bwd_mask_TBps"] = round(mb * 4 / rec["bwd_mask_us"], 3)
            rec["bwd_mask_nodres_us"] = round(timed(bwdm_nodres, args.reps), 2)
            rec["bwd_mask_nodres_TBps"] = round(mb * 3 / rec["bwd_mask_nodres_us"], 3)
        if relu and not res and not args.unfused:
            t = timed(bwd(False), args.reps)
            rec["bwd_remask_us"] = round(t, 2)
            rec["bwd_remask_TBps"] = round(mb * 3 / t, 3)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
