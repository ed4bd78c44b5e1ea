"""The convs whose GEMMs run 64- or 32-row tiles (M <= 64: the 19-class ASPP heads, layer1's
64-channel 3x3) in each fp32 form, fwd and fwd+bwd per op call (HIP events, 20 calls after
warm-up): bf16x6 keeps them on exact f32 MFMA, f16x3 on the per-read fp16 split (kMathH3)."""
import json
import sys

import torch

sys.path.insert(0, ".")
from maxsquareloss_amd import ops  # noqa: E402


def t(fn, iters=20):
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


def run(form):
    ops.set_f32_form(form)
    torch.manual_seed(0)
    for name, cin, cout, h, w, d, nb in [("aspp6", 2048, 19, 65, 129, 6, 2), ("aspp5", 1024, 19, 65, 129, 6, 2),
                                          ("l1_3x3", 64, 64, 129, 257, 1, 1)]:
        x = torch.relu(torch.randn(1, cin, h, w, device="cuda")).requires_grad_()
        w0 = (torch.randn(cout, cin, 3, 3, device="cuda") * 0.01).requires_grad_()
        w1 = (torch.randn(cout, cin, 3, 3, device="cuda") * 0.01).requires_grad_()
        b0 = torch.zeros(cout, device="cuda", requires_grad=True)
        b1 = torch.zeros(cout, device="cuda", requires_grad=True)
        gy = torch.randn(1, cout, h, w, device="cuda") * 1e-3
        cache = ops.PackCache()
        if nb == 2:
            f = lambda: ops.aspp2(x, w0, b0, w1, b1, 6, 12, cache)
        else:
            f = lambda: ops.dconv3x3(x, w0, d, cache)
        with torch.no_grad():
            fwd = t(f)
        y = f()
        bwd = t(lambda: torch.autograd.grad(y, [x, w0] if nb == 1 else [x, w0, w1, b0, b1], gy, retain_graph=True))
        print(json.dumps({"form": form, "op": name, "fwd_us": round(fwd, 1), "bwd_us": round(bwd, 1)}), flush=True)


if __name__ == "__main__":
    for form in (sys.argv[1] if len(sys.argv) > 1 else "bf16x6,f16x3,bf16x6,f16x3").split(","):
        run(form)
