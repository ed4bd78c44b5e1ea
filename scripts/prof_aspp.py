"""The layer6 ASPP head alone (2048 -> 19 classes, d = 6 / 12, shift form: Z = W'x pointwise GEMM, masked
shift-add; backward: gathered dY, dx = W'^T G, dW' = G x^T) over the image pair at the 1024x512 feature
size, forward + backward, launched through the same op as the training step.  Profiled by
scripts/gpu_counters.sh (one --pmc pass per counter group) for the r04 ASPP traffic evidence.

    prof_aspp.py [N] [H W]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from maxsquareloss_amd import ops  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
H, W = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (65, 129)
g = torch.Generator(device="cuda").manual_seed(0)
x = torch.randn((1, 2048, 2, H, W), device="cuda", generator=g).requires_grad_()
w0 = (torch.randn(19, 2048, 3, 3, device="cuda", generator=g) * 0.01).requires_grad_()
w1 = (torch.randn(19, 2048, 3, 3, device="cuda", generator=g) * 0.01).requires_grad_()
b0 = torch.zeros(19, device="cuda", requires_grad=True)
b1 = torch.zeros(19, device="cuda", requires_grad=True)
gy = torch.randn((1, 19, 2, H, W), device="cuda", generator=g)
cache = ops.PackCache()
for _ in range(n):
    y = ops.aspp2(x, w0, b0, w1, b1, 6, 12, cache)
    y.backward(gy)
torch.cuda.synchronize()
print("iterations", n, "checksum", float(y.double().sum()), float(x.grad.double().abs().sum()))
