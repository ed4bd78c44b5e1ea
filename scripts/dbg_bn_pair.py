"""Debug (r05): the fused BN forward on an image pair vs two single-image calls, via the C-ABI - which of
save_mean / save_invstd / y / running stats differ, and by how many ulps."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from maxsquareloss_amd import hip  # noqa: E402

lib = hip.load()
c, h, w = 256, 65, 129
p = h * w
g = torch.Generator().manual_seed(c + h)
x = (torch.randn(1, c, 2, h, w, generator=g) * 3 + 1).cuda()
r = torch.randn(1, c, 2, h, w, generator=g).cuda()
gam = torch.rand(c, generator=g).cuda() + 0.5
bet = torch.randn(c, generator=g).cuda()
rm0 = torch.randn(c, generator=g).cuda()
rv0 = torch.ones(c).cuda()


def run(xx, rr, n, rm, rv, nb):
    y = torch.empty_like(xx)
    sm = torch.empty(c * n, device="cuda")
    si = torch.empty(c * n, device="cuda")
    ws = hip.workspace(lib.msl_bn_workspace(c, p, n), "cuda")
    hip.check(lib.msl_bn_fwd(xx.data_ptr(), gam.data_ptr(), bet.data_ptr(), rr.data_ptr(), y.data_ptr(), rm.data_ptr(),
                             rv.data_ptr(), nb.data_ptr(), sm.data_ptr(), si.data_ptr(), c, p, n, 1, 1, 0.1, 1e-5, 1,
                             ws.data_ptr(), ws.numel(), hip.stream_ptr()), "bn")
    return y, sm, si


rmA, rvA, nbA = rm0.clone(), rv0.clone(), torch.zeros(1, dtype=torch.int64, device="cuda")
yA, smA, siA = run(x, r, 2, rmA, rvA, nbA)
rmB, rvB, nbB = rm0.clone(), rv0.clone(), torch.zeros(1, dtype=torch.int64, device="cuda")
outs = [run(x[:, :, i].contiguous(), r[:, :, i].contiguous(), 1, rmB, rvB, nbB) for i in range(2)]
torch.cuda.synchronize()
smB = torch.stack([o[1] for o in outs], 1).reshape(-1)
siB = torch.stack([o[2] for o in outs], 1).reshape(-1)


def ulps(a, b):
    return (a.view(torch.int32).long() - b.view(torch.int32).long()).abs()


print("save_mean differ", int((ulps(smA, smB) > 0).sum()), "max ulp", int(ulps(smA, smB).max()))
print("save_invstd differ", int((ulps(siA, siB) > 0).sum()), "max ulp", int(ulps(siA, siB).max()))
print("y differ", int((yA[:, :, 0] != outs[0][0]).sum()), int((yA[:, :, 1] != outs[1][0]).sum()))
print("running_mean differ", int((ulps(rmA, rmB) > 0).sum()), "max ulp", int(ulps(rmA, rmB).max()))
print("running_var differ", int((ulps(rvA, rvB) > 0).sum()), "max ulp", int(ulps(rvA, rvB).max()))
print("num_batches", int(nbA), int(nbB))
k = int(ulps(rmA, rmB).argmax())
print("channel", k, "rmA", rmA[k].item(), "rmB", rmB[k].item(), "means pair", smA[2 * k].item(), smA[2 * k + 1].item(),
      "single", smB[2 * k].item(), smB[2 * k + 1].item(), "rm0", rm0[k].item())
