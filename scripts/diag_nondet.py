"""Find the first nondeterministic op of the backward: two identical forward/backward passes of
DeeplabMulti (train mode), the gradient at every module output captured by hooks, compared in
backward order (the first module whose output gradient matches but whose input-side differs is
the culprit)."""
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
for _ in range(2):  # warm-up: MIOpen's first calls may pick other kernels
    x2, x1 = model(x)
    (x2.square().mean() + 0.1 * x1.square().mean()).backward()
torch.cuda.synchronize()
runs = []
for k in range(2):
    grads = []

    def mk(name):
        def fwd_hook(mod, inp, out):
            t = out[0] if isinstance(out, tuple) else out
            if t.requires_grad:
                t.register_hook(lambda g, n=name: grads.append((n, g.detach().clone())))
        return fwd_hook

    hs = [m.register_forward_hook(mk(n)) for n, m in model.named_modules() if n]
    for p in model.parameters():
        p.grad = None
    x2, x1 = model(x)
    x2.register_hook(lambda g: grads.insert(0, ("x2 (model output)", g.detach().clone())))
    (x2.square().mean() + 0.1 * x1.square().mean()).backward()
    torch.cuda.synchronize()
    for h in hs:
        h.remove()
    runs.append(grads)
a, b = runs
print("hooked gradients", len(a), len(b), flush=True)
first = None
for (na, ga), (nb, gb) in zip(a, b):
    same = torch.equal(ga, gb)
    if not same and first is None:
        first = na
        d = (ga - gb).abs().max().item() / max(ga.abs().max().item(), 1e-30)
        print("first differing output gradient (backward order):", na, "rel", d, flush=True)
idx = [n for n, _ in a].index(first) if first else -1
print("context (backward order):", [n for n, _ in a][max(0, idx - 4):idx + 3], flush=True)
print("x2 grad equal:", torch.equal(a[0][1], b[0][1]), a[0][0], flush=True)
