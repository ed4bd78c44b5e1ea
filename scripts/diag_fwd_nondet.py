"""First module whose forward output differs between two identical train-mode forwards of
DeeplabMulti (after two warm-up passes), in forward order."""
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
with torch.no_grad():
    for _ in range(2):
        model(x)
runs = []
for k in range(2):
    outs = []
    hs = [m.register_forward_hook(lambda mod, i, o, n=n: outs.append((n, (o[0] if isinstance(o, tuple) else o).detach().clone())))
          for n, m in model.named_modules() if n]
    with torch.no_grad():
        model(x)
    torch.cuda.synchronize()
    for h in hs:
        h.remove()
    runs.append(outs)
nd = 0
for (na, a), (nb, b) in zip(*runs):
    if not torch.equal(a, b):
        d = (a - b).abs().max().item() / max(a.abs().max().item(), 1e-30)
        print("differs:", na, tuple(a.shape), "rel", d, flush=True)
        nd += 1
        if nd >= 6:
            break
print("modules compared", len(runs[0]), "differing shown", nd, flush=True)
