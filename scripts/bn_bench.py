"""A/B of the BN kernel forms (msl_bn_set_fused) on the model's train-mode shapes at 1024x512:
fwd and fwd+bwd per call, HIP events on torch's stream (the ops launch there)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from maxsquareloss_amd import ops

SHAPES = [(64, 129, 257, False, True), (256, 129, 257, True, True), (256, 65, 129, False, True), (1024, 65, 129, True, True),
          (512, 65, 129, False, True), (2048, 65, 129, True, True), (128, 65, 129, False, True)]


def run(c, h, w, res, relu, fused, it=50):
    ops.set_bn_fused(fused)
    bn = torch.nn.BatchNorm2d(c).cuda().train()
    x = (torch.randn(1, c, h, w, device="cuda") * 3 + 4).requires_grad_()
    r = torch.randn(1, c, h, w, device="cuda").requires_grad_() if res else None
    gy = torch.randn(1, c, h, w, device="cuda")
    for _ in range(5):
        ops.bn_act(bn, x, residual=r, relu=relu).backward(gy)
    e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    torch.cuda.synchronize()
    tf = tb = 0.0
    for _ in range(it):
        e[0].record()
        y = ops.bn_act(bn, x, residual=r, relu=relu)
        e[1].record()
        y.backward(gy)
        e[2].record()
        torch.cuda.synchronize()
        tf += e[0].elapsed_time(e[1])
        tb += e[1].elapsed_time(e[2])
    mb = c * h * w * 4 / 1e6
    return tf / it * 1e3, tb / it * 1e3, mb


for s in SHAPES:
    a = run(*s, fused=False)
    b = run(*s, fused=True)
    print(f"c={s[0]:5d} p={s[1]*s[2]:6d} res={int(s[3])} {a[2]:6.1f} MB  split fwd {a[0]:6.1f} bwd {a[1]:6.1f} us"
          f"  | fused fwd {b[0]:6.1f} bwd {b[1]:6.1f} us", flush=True)
