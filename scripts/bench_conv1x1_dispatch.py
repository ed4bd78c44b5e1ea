"""Per-GEMM timing of every stride-1 1x1 conv of the model (1024x512 input): each of the three GEMMs
(y = W x, dx = W^T dy, dW += dy x^T) on every implementation available - MIOpen, hipBLASLt
(torch.mm / addmm_) and the HIP pointwise kernels (hip_x6 = the split fp32 form in use: bf16x6 or f16x3) - weighted by how often the UDA step runs
it.  Prints the per-GEMM winners as the dispatch table of ops._Conv1x1 (profiles/)."""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from maxsquareloss_amd import hip, ops  # noqa: E402

# (cin, cout, h, w): uses per UDA iteration (2 images)
SHAPES = {(64, 64, 129, 257): 2, (64, 256, 129, 257): 8, (256, 64, 129, 257): 4,
          (128, 512, 65, 129): 8, (512, 128, 65, 129): 6,
          (512, 256, 65, 129): 2, (512, 1024, 65, 129): 2, (256, 1024, 65, 129): 46, (1024, 256, 65, 129): 44,
          (1024, 512, 65, 129): 2, (1024, 2048, 65, 129): 2, (512, 2048, 65, 129): 6, (2048, 512, 65, 129): 4}


def t(fn, iters=15):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    lib = hip.load()
    if "--sk-hybrid" in sys.argv:  # A/B of the forward-form schedule (msl_conv_set_sk_hybrid)
        hip.check(lib.msl_conv_set_sk_hybrid(int(sys.argv[sys.argv.index("--sk-hybrid") + 1])), "sk_hybrid")
    if "--form" in sys.argv:  # the fp32 form of the HIP kernels (default: the library's)
        ops.set_f32_form(sys.argv[sys.argv.index("--form") + 1])
    print(f"fp32 form of the HIP GEMMs: {ops.f32_form()} (f16x3: the operands' absmax partials computed once, "
          "outside the timed calls, as the BN kernels hand them over in the step)", flush=True)
    table, tot = {}, {"lib": 0.0, "best": 0.0}
    for (cin, cout, h, w), n in SHAPES.items():
        p = h * w
        x = torch.randn(1, cin, h, w, device="cuda")
        wt = torch.randn(cout, cin, 1, 1, device="cuda") * 0.05
        gy = torch.randn(1, cout, h, w, device="cuda")
        x2, g2, w2 = x.view(cin, p), gy.view(cout, p), wt.view(cout, cin)
        cache = ops.PackCache(pointwise=True)
        packed, packed_d = cache.get([wt], cin, cout, 0), cache.get([wt], cin, cout, 1)
        s = hip.stream_ptr()
        ctr = hip.counters(x.device).data_ptr()
        wsf = hip.workspace(lib.msl_pconv_fwd_workspace(cin, cout, p), x.device)
        wsd = hip.workspace(lib.msl_pconv_dgrad_workspace(cin, cout, p), x.device)
        wsw = hip.workspace(lib.msl_pconv_wgrad_workspace(cin, cout, p), x.device)
        y, dx, dw = torch.empty(1, cout, h, w, device="cuda"), torch.empty_like(x), torch.zeros_like(wt)
        npart = lib.msl_absmax_parts()
        xp, gp = torch.empty(npart, device="cuda"), torch.empty(npart, device="cuda")
        lib.msl_absmax_partials(x.data_ptr(), x.numel(), xp.data_ptr(), s)
        lib.msl_absmax_partials(gy.data_ptr(), gy.numel(), gp.data_ptr(), s)
        r = {}
        r["fwd"] = {
            "miopen": t(lambda: F.conv2d(x, wt)),
            "hipblaslt": t(lambda: torch.mm(w2, x2)),
            "hip_x6": t(lambda: lib.msl_pconv_fwd_sc(x.data_ptr(), packed.data_ptr(), y.data_ptr(), cin, cout, p, ctr,
                                                     wsf.data_ptr(), wsf.numel(), s, xp.data_ptr(), npart)),
        }
        r["dgrad"] = {
            "miopen": t(lambda: torch.ops.aten.convolution_backward(gy, x, wt, None, (1, 1), (0, 0), (1, 1), False,
                                                                     (0, 0), 1, (True, False, False))),
            "hipblaslt": t(lambda: torch.mm(w2.t(), g2)),
            "hip_x6": t(lambda: lib.msl_pconv_dgrad_acc_sc(gy.data_ptr(), packed_d.data_ptr(), dx.data_ptr(), cin, cout,
                                                           p, 0, ctr, wsd.data_ptr(), wsd.numel(), s, gp.data_ptr(),
                                                           npart)),
        }
        r["wgrad"] = {
            "hipblaslt": t(lambda: dw.view(cout, cin).addmm_(g2, x2.t())),
            "hip_x6": t(lambda: lib.msl_pconv_wgrad_sc(x.data_ptr(), gy.data_ptr(), dw.data_ptr(), cin, cout, p, 1,
                                                       wsw.data_ptr(), wsw.numel(), s, xp.data_ptr(), npart,
                                                       gp.data_ptr(), npart)),
        }
        # dx += W^T dy (the identity residual's gradient summed by the data-gradient GEMM,
        # ops.ResidualGrad): separate add after MIOpen vs the accumulating GEMMs
        res = torch.zeros_like(x)
        acc = {
            "miopen+add": t(lambda: res.add_(torch.ops.aten.convolution_backward(
                gy, x, wt, None, (1, 1), (0, 0), (1, 1), False, (0, 0), 1, (True, False, False))[0])),
            "hipblaslt_addmm": t(lambda: res.view(cin, p).addmm_(w2.t(), g2)),
            "hip_x6_acc": t(lambda: lib.msl_pconv_dgrad_acc_sc(gy.data_ptr(), packed_d.data_ptr(), res.data_ptr(), cin,
                                                               cout, p, 1, ctr, wsd.data_ptr(), wsd.numel(), s,
                                                               gp.data_ptr(), npart)),
        }
        pack = t(lambda: (lib.msl_pconv_pack(wt.data_ptr(), cin, cout, 0, packed.data_ptr(), s),
                          lib.msl_pconv_pack(wt.data_ptr(), cin, cout, 1, packed_d.data_ptr(), s)))
        best = {k: min(v, key=v.get) for k, v in r.items()}
        cur = r["fwd"]["miopen"] + min(r["dgrad"]["miopen"], r["dgrad"]["hipblaslt"]) + r["wgrad"]["hipblaslt"]
        bst = sum(r[k][best[k]] for k in r) + (pack / 2 if "hip_x6" in best.values() else 0.0)  # one pack per step
        tot["lib"] += n * cur
        tot["best"] += n * bst
        key = f"{cin}x{cout}x{p}"
        table[key] = best
        print(f"{cin:5d}->{cout:5d} P {p:6d} x{n:2d} | " + " | ".join(
            f"{k}: " + " ".join(f"{m} {v:6.1f}" for m, v in r[k].items()) for k in r) + f" | packs {pack:5.1f} | best {best}",
            flush=True)
        print("        dgrad accumulating into the residual gradient: " +
              " ".join(f"{m} {v:6.1f}" for m, v in acc.items()), flush=True)
    print(f"per UDA step: library mix {tot['lib'] / 1e3:.2f} ms, per-GEMM best {tot['best'] / 1e3:.2f} ms", flush=True)
    print("TABLE " + json.dumps(table), flush=True)


if __name__ == "__main__":
    main()
