"""Whole-model gradients with the fused residual gradient vs autograd's accumulation: one
forward/backward of DeeplabMulti (train mode) at HxW, every parameter gradient compared
normwise; --baseline compares two unfused passes (the run-to-run spread)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from maxsquareloss_amd.graphs.models import deeplab_multi as dm  # noqa: E402
from maxsquareloss_amd.utils.synthetic import synthetic_image  # noqa: E402

H, W = int(sys.argv[1]), int(sys.argv[2])
torch.manual_seed(0)
model = dm.DeeplabMulti(num_classes=19, pretrained=False).cuda().train()
x = synthetic_image(H, W, 3).cuda()
res = {}
for _ in range(2):  # settle MIOpen's solver choice (its first calls may pick other kernels)
    x2, x1 = model(x)
    (x2.square().mean() + 0.1 * x1.square().mean()).backward()
torch.cuda.synchronize()
modes = (False, False) if "--baseline" in sys.argv else (False, True)
for k, fuse in enumerate(modes):
    dm.PointwiseConv.fuses_residual_grad = (lambda self, f=fuse: f)
    for p in model.parameters():
        p.grad = None
    x2, x1 = model(x)
    (x2.square().mean() + 0.1 * x1.square().mean()).backward()
    torch.cuda.synchronize()
    res[k] = {n: p.grad.detach().double().clone() for n, p in model.named_parameters() if p.grad is not None}
worst = []
for n, g in res[0].items():
    d = (res[1][n] - g).norm().item() / max(g.norm().item(), 1e-30)
    worst.append((d, n))
worst.sort(reverse=True)
print("modes", modes, "max rel diff", worst[0][0], flush=True)
for d, n in worst[:8]:
    print(f"  {d:.3e} {n}", flush=True)
