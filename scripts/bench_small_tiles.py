"""Times the ops that run on 64- / 32-row tiles (the ASPP heads, 19 classes; the 64-channel layer1
3x3 convs): forward and backward, fp32 form bf16x6 (profiles/r02_small_tile_x6.txt: the x6 kernels on
those tiles were tried and not adopted)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from maxsquareloss_amd import ops  # noqa: E402


def t(fn, iters=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    ops.set_f32_form("bf16x6")
    dev = "cuda"
    for cin in (1024, 2048):
        x = torch.randn(1, cin, 65, 129, device=dev, requires_grad=True)
        w0 = (torch.randn(19, cin, 3, 3, device=dev) * 0.01).requires_grad_()
        w1 = (torch.randn(19, cin, 3, 3, device=dev) * 0.01).requires_grad_()
        b0 = torch.zeros(19, device=dev, requires_grad=True)
        b1 = torch.zeros(19, device=dev, requires_grad=True)
        cache = ops.PackCache()
        f = lambda: ops.aspp2(x, w0, b0, w1, b1, 6, 12, cache)  # noqa: E731
        y = f()
        gy = torch.randn_like(y)
        tf = t(lambda: f())
        tb = t(lambda: torch.autograd.grad(f(), (x, w0, w1, b0, b1), gy)) - tf
        print(f"aspp {cin}->19 65x129: fwd {tf:7.1f} us  bwd {tb:7.1f} us", flush=True)
    x = torch.randn(1, 64, 129, 257, device=dev, requires_grad=True)
    w = (torch.randn(64, 64, 3, 3, device=dev) * 0.05).requires_grad_()
    cache = ops.PackCache()
    f = lambda: ops.dconv3x3(x, w, 1, cache)  # noqa: E731
    gy = torch.randn_like(f())
    tf = t(lambda: f())
    tb = t(lambda: torch.autograd.grad(f(), (x, w), gy)) - tf
    print(f"dconv 64->64 129x257 d1: fwd {tf:7.1f} us  bwd {tb:7.1f} us", flush=True)


if __name__ == "__main__":
    main()
