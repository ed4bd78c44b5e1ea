import sys; sys.path.insert(0, ".")
import torch
from maxsquareloss_amd import ops
c, h, w = 256, 65, 129
g = torch.Generator().manual_seed(c + h)
x = torch.randn(1, c, h, w, generator=g) * 3 + 40.0
r = torch.randn(1, c, h, w, generator=g)
gamma = torch.rand(c, generator=g) + 0.5
beta = torch.randn(c, generator=g)
rm, rv = torch.randn(c, generator=g), torch.rand(c, generator=g) + 0.5
gy = torch.randn(1, c, h, w, generator=g)
bn = torch.nn.BatchNorm2d(c).cuda()
with torch.no_grad():
    bn.weight.copy_(gamma); bn.bias.copy_(beta); bn.running_mean.copy_(rm); bn.running_var.copy_(rv)
xr = x.double().requires_grad_(); rr = r.double().requires_grad_()
yr = torch.relu(torch.nn.functional.batch_norm(xr, rm.double(), rv.double(), gamma.double(), beta.double(), True, 0.1, 1e-5) + rr)
yr.backward(gy.double())
xg = x.cuda().requires_grad_(); rg = r.cuda().requires_grad_()
y = ops.bn_act(bn, xg, residual=rg, relu=True)
y.backward(gy.cuda())
d = (xg.grad.double().cpu() - xr.grad).abs()
i = torch.argmax(d).item()
cc, p = divmod(i, h * w)
print("max err", d.max().item(), "at ch", cc, "p", p, "ours", xg.grad.view(-1)[i].item(), "ref", xr.grad.view(-1)[i].item())
print("y ours", y.view(-1)[i].item(), "ref", yr.view(-1)[i].item(), "gy", gy.view(-1)[i].item())
dc = d[0, cc]
print("channel max err", dc.max().item(), "mean err", dc.mean().item(), "max ref", xr.grad[0, cc].abs().max().item())
mask_ours = (y.detach().cpu() > 0); mask_ref = (yr.detach() > 0)
print("mask flips", (mask_ours != mask_ref).sum().item(), "in channel", (mask_ours[0, cc] != mask_ref[0, cc]).sum().item())
print("dres err", (rg.grad.double().cpu() - rr.grad).abs().max().item())
