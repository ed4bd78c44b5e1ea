"""Forward / data-gradient outputs of the forward-form conv GEMMs at the step's shapes, saved for a
bitwise comparison of two library builds (MSL_LIB_PATH) or settings that must agree bit for bit
(r04: k_sk_reduce vs an in-launch fix-up of split stream-K tiles, profiles/r04_sk_fixup_ab.txt).

    fix_parity.py save OUT.pt        fix_parity.py compare A.pt B.pt"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

if sys.argv[1] == "compare":
    a, b = torch.load(sys.argv[2], weights_only=True), torch.load(sys.argv[3], weights_only=True)
    bad = [k for k in a if not torch.equal(a[k], b[k])]
    for k in a:
        print(f"{k:40s} {'DIFFERENT' if k in bad else 'bit-identical'}")
    sys.exit(1 if bad else 0)

from maxsquareloss_amd import ops  # noqa: E402

torch.manual_seed(0)
dev = "cuda"
out = {}
for nimg in (1, 2):
    for (cin, cout, h, w, d) in [(256, 256, 65, 129, 2), (64, 64, 129, 257, 1), (512, 512, 65, 129, 4),
                                 (2048, 19, 65, 129, 6)]:
        x = torch.randn(1, cin, nimg, h, w, device=dev).requires_grad_()
        wt = torch.randn(cout, cin, 3, 3, device=dev) * 0.02
        y = ops.dconv3x3(x, wt, d, ops.PackCache())
        y.backward(torch.randn_like(y))
        out[f"dconv {cin}->{cout} d{d} n{nimg} y"] = y.detach().cpu()
        out[f"dconv {cin}->{cout} d{d} n{nimg} dx"] = x.grad.cpu()
    for (cin, cout, h, w) in [(1024, 256, 65, 129), (256, 1024, 65, 129), (2048, 512, 65, 129), (64, 256, 129, 257)]:
        x = torch.randn(1, cin, nimg, h, w, device=dev).requires_grad_()
        wt = torch.randn(cout, cin, 1, 1, device=dev) * 0.02
        y = ops.pconv(x, wt, ops.PackCache(pointwise=True))
        y.backward(torch.randn_like(y))
        out[f"pconv {cin}->{cout} n{nimg} y"] = y.detach().cpu()
        out[f"pconv {cin}->{cout} n{nimg} dx"] = x.grad.cpu()
torch.save(out, sys.argv[2])
print(len(out), "tensors saved")
