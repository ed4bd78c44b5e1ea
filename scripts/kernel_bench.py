"""Per-kernel timing of the hot-path HIP ops vs PyTorch-ROCm (MIOpen) at the 1024x512 shapes.

Prints one JSON line per op: ms per call and TFLOP/s (algorithmic FLOPs).
"""
import json
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from maxsquareloss_amd import ops  # noqa: E402


def timeit(fn, iters=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def conv_case(name, cin, cout, h, w, d):
    x = torch.randn(1, cin, h, w, device="cuda")
    wt = (torch.randn(cout, cin, 3, 3, device="cuda") * 0.01).requires_grad_()
    gy = torch.randn(1, cout, h, w, device="cuda")
    flops = 2.0 * cin * cout * 9 * h * w
    cache = ops.PackCache()
    xg = x.clone().requires_grad_()
    res = {"op": name, "shape": [cin, cout, h, w, d]}
    res["hip_fwd_ms"] = timeit(lambda: ops.dconv3x3(x, wt.detach(), d, cache))
    y = ops.dconv3x3(xg, wt, d, cache)

    def bwd():
        xg.grad = None
        wt.grad = None
        torch.autograd.grad(y, [xg, wt], gy, retain_graph=True)
    res["hip_bwd_ms"] = timeit(bwd)
    res["torch_fwd_ms"] = timeit(lambda: F.conv2d(x, wt.detach(), padding=d, dilation=d))
    yt = F.conv2d(xg, wt, padding=d, dilation=d)
    res["torch_bwd_ms"] = timeit(lambda: torch.autograd.grad(yt, [xg, wt], gy, retain_graph=True))
    res["hip_fwd_tflops"] = flops / res["hip_fwd_ms"] / 1e9
    res["hip_bwd_tflops"] = 2 * flops / res["hip_bwd_ms"] / 1e9
    res["torch_fwd_tflops"] = flops / res["torch_fwd_ms"] / 1e9
    res["torch_bwd_tflops"] = 2 * flops / res["torch_bwd_ms"] / 1e9
    print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in res.items()}), flush=True)


def aspp_case(name, cin, c, h, w):
    x = torch.randn(1, cin, h, w, device="cuda")
    w0 = (torch.randn(c, cin, 3, 3, device="cuda") * 0.01).requires_grad_()
    w1 = (torch.randn(c, cin, 3, 3, device="cuda") * 0.01).requires_grad_()
    b0 = torch.zeros(c, device="cuda", requires_grad=True)
    b1 = torch.zeros(c, device="cuda", requires_grad=True)
    gy = torch.randn(1, c, h, w, device="cuda")
    flops = 2 * 2.0 * cin * c * 9 * h * w
    cache = ops.PackCache()
    xg = x.clone().requires_grad_()
    res = {"op": name, "shape": [cin, c, h, w]}
    res["hip_fwd_ms"] = timeit(lambda: ops.aspp2(x, w0.detach(), b0.detach(), w1.detach(), b1.detach(), 6, 12, cache))
    y = ops.aspp2(xg, w0, b0, w1, b1, 6, 12, cache)
    res["hip_bwd_ms"] = timeit(lambda: torch.autograd.grad(y, [xg, w0, w1, b0, b1], gy, retain_graph=True))
    res["torch_fwd_ms"] = timeit(lambda: F.conv2d(x, w0, b0, padding=6, dilation=6) + F.conv2d(x, w1, b1, padding=12, dilation=12))
    yt = F.conv2d(xg, w0, b0, padding=6, dilation=6) + F.conv2d(xg, w1, b1, padding=12, dilation=12)
    res["torch_bwd_ms"] = timeit(lambda: torch.autograd.grad(yt, [xg, w0, w1, b0, b1], gy, retain_graph=True))
    res["hip_fwd_tflops"] = flops / res["hip_fwd_ms"] / 1e9
    res["hip_bwd_tflops"] = 2 * flops / res["hip_bwd_ms"] / 1e9
    print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in res.items()}), flush=True)


def loss_case():
    low = torch.randn(1, 19, 65, 129, device="cuda", requires_grad=True)
    y = torch.randint(-1, 19, (512 * 1024,), device="cuda")
    res = {"op": "losses_1024x512"}
    res["upsample_fwd_ms"] = timeit(lambda: ops.upsample_bilinear(low.detach(), (512, 1024)))
    res["ce_fwd_ms"] = timeit(lambda: ops.ce_up(low.detach(), y, (512, 1024)))
    l = ops.ce_up(low, y, (512, 1024))
    res["ce_bwd_ms"] = timeit(lambda: torch.autograd.grad(l, [low], retain_graph=True))
    l = ops.maxsquare_up(low, (512, 1024))
    res["ms_fwd_ms"] = timeit(lambda: ops.maxsquare_up(low.detach(), (512, 1024)))
    res["ms_bwd_ms"] = timeit(lambda: torch.autograd.grad(l, [low], retain_graph=True))
    res["iw_fwd_ms"] = timeit(lambda: ops.iw_maxsquare_up(low.detach(), (512, 1024), 0.2))
    up = F.interpolate(low.detach(), size=(512, 1024), mode="bilinear", align_corners=True)
    res["torch_softmax_ms_fwd"] = timeit(lambda: F.softmax(up, 1))
    print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in res.items()}), flush=True)


if __name__ == "__main__":
    torch.manual_seed(0)
    conv_case("a1_layer3_d2", 256, 256, 65, 129, 2)
    conv_case("a2_layer4_d4", 512, 512, 65, 129, 4)
    conv_case("layer1_d1", 64, 64, 129, 257, 1)
    conv_case("layer2_d1", 128, 128, 65, 129, 1)
    aspp_case("a3_layer5", 1024, 19, 65, 129)
    aspp_case("a3_layer6", 2048, 19, 65, 129)
    loss_case()
