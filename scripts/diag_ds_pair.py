"""layer2.0.downsample.0 at the model's shapes: stride-2 256 -> 512 pointwise conv (shared subsample) on a
pair and on one image, every fp32 form, y / dx / dW against fp64 (sink into a flat-buffer slice and plain)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from maxsquareloss_amd import ops  # noqa: E402


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return (a - b).abs().max().item() / max(b.abs().max().item(), 1e-30)


def case(nimg, H, W, cin, cout, form):
    prev = ops.set_f32_form(form)
    g = torch.Generator().manual_seed(7)
    shape = (1, cin, nimg, H, W) if nimg > 1 else (1, cin, H, W)
    x = torch.relu(torch.randn(shape, generator=g))
    wt = torch.randn(cout, cin, 1, 1, generator=g) * 0.05
    ho, wo = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    oshape = (1, cout, nimg, ho, wo) if nimg > 1 else (1, cout, ho, wo)
    gy = torch.randn(oshape, generator=g)
    xg = x.cuda().requires_grad_()
    wg = wt.cuda().requires_grad_()
    cache = ops.PackCache(pointwise=True)
    xs = ops.subsample(xg, 2)
    y = ops.pconv(xs, wg, cache)
    y.backward(gy.cuda())
    torch.cuda.synchronize()
    wr = wt.double().requires_grad_()
    dwr = torch.zeros_like(wr)
    out = []
    for i in range(nimg):
        xi = (x[:, :, i] if nimg > 1 else x).double().requires_grad_()
        yi = F.conv2d(xi, wr, stride=2)
        gi = (gy[:, :, i] if nimg > 1 else gy).double()
        yi.backward(gi)
        yg = y[:, :, i] if nimg > 1 else y
        dxg = xg.grad[:, :, i] if nimg > 1 else xg.grad
        out.append((rel(yg, yi), rel(dxg, xi.grad)))
    r = rel(wg.grad, wr.grad)
    ops.set_f32_form(prev)
    return out, r


for form in ("f16x3", "mfma_f32", "bf16x6"):
    for nimg, H, W in ((2, 65, 129), (1, 65, 129), (2, 129, 257), (1, 129, 257)):
        per, r = case(nimg, H, W, 256, 512, form)
        print(f"{form} nimg {nimg} {H}x{W}: y/dx per image {[(f'{a:.1e}', f'{b:.1e}') for a, b in per]} dW {r:.2e}",
              flush=True)
