"""Accuracy of the fp32 conv forms against fp64 (profiles/r02_f16x3_accuracy.txt): per output element,
|out - fp64| / (the same conv of |operands|) - the error relative to the element's own sum of
|terms| - max and mean over the tensor, for fwd / data gradient / weight gradient, on the layer3
and layer4 dilated shapes at 1024x512 with unit-scale and far-out-of-fp16-range operands."""
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from maxsquareloss_amd import ops  # noqa: E402


def errs(out, ref, bound):
    e = (out.detach().double().cpu() - ref) / bound.clamp_min(1e-300)
    return e.abs().max().item(), e.abs().mean().item()


for cin, cout, h, w, d in [(256, 256, 65, 129, 2), (512, 512, 65, 129, 4)]:
    for xs, gs in [(1.0, 1e-6), (1e-20, 1e15)]:
        g = torch.Generator().manual_seed(cin + h)
        x = torch.relu(torch.randn(1, cin, h, w, generator=g)) * xs
        wt = torch.randn(cout, cin, 3, 3, generator=g) * 0.01
        gy = torch.randn(1, cout, h, w, generator=g) * gs
        xr, wr = x.double().requires_grad_(), wt.double().requires_grad_()
        yr = F.conv2d(xr, wr, padding=d, dilation=d)
        yr.backward(gy.double())
        xa, wa = x.double().abs().requires_grad_(), wt.double().abs().requires_grad_()
        ya = F.conv2d(xa, wa, padding=d, dilation=d)
        ya.backward(gy.double().abs())
        for form in ("mfma_f32", "bf16x6", "f16x3"):
            prev = ops.set_f32_form(form)
            xg, wg = x.cuda().requires_grad_(), wt.cuda().requires_grad_()
            y = ops.dconv3x3(xg, wg, d, ops.PackCache())
            y.backward(gy.cuda())
            torch.cuda.synchronize()
            r = [errs(y, yr.detach(), ya.detach()), errs(xg.grad, xr.grad, xa.grad), errs(wg.grad, wr.grad, wa.grad)]
            ops.set_f32_form(prev)
            print(f"{cin}->{cout} d={d} x*{xs:g} dy*{gs:g} {form:9s} "
                  + "  ".join(f"{k} max {m:.2e} mean {a:.2e}" for k, (m, a) in zip(("fwd", "dgrad", "wgrad"), r)),
                  flush=True)
