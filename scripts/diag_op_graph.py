"""Isolate the captured-step mismatch of layer2.0.downsample.0.weight: the stride-2 256 -> 512 pointwise
conv (swapped-operand f16x3 weight gradient) on a pair-shaped input, eager vs inside a captured hipGraph,
both against fp64, with the weight gradient accumulated into a flat-buffer slice (the trainer's sink) or
returned.  Also the same op with the subsample and a BN after it (the block's downsample branch)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

from maxsquareloss_amd import ops  # noqa: E402


def run_case(nimg, h, w, cin, cout, graph, use_bn):
    g = torch.Generator().manual_seed(5)
    shape = (1, cin, nimg, 2 * h - 1, 2 * w - 1) if nimg > 1 else (1, cin, 2 * h - 1, 2 * w - 1)
    x0 = torch.relu(torch.randn(shape, generator=g)).cuda()
    wt = (torch.randn(cout, cin, 1, 1, generator=g) * 0.05).cuda().requires_grad_()
    oshape = (1, cout, nimg, h, w) if nimg > 1 else (1, cout, h, w)
    gy = torch.randn(oshape, generator=g).cuda()
    bn = nn.BatchNorm2d(cout).cuda().train()
    pack = ops.PackCache(pointwise=True)

    def body():
        xs = ops.subsample(x0, 2)
        y = ops.pconv(xs, wt, pack)
        if use_bn:
            y = ops.bn_act(bn, y)
        y.backward(gy)

    def once():
        wt.grad = None
        if graph:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                body()  # warm-up (eager)
            torch.cuda.current_stream().wait_stream(s)
            torch.cuda.synchronize()
            wt.grad = None
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr, stream=s):
                body()
            held = wt.grad
            gr.replay()
            torch.cuda.synchronize()
            return held.detach().clone()
        body()
        torch.cuda.synchronize()
        return wt.grad.detach().clone()

    return once()


for nimg, use_bn in ((2, False), (2, True), (1, False), (1, True)):
    e = run_case(nimg, 33, 65, 256, 512, False, use_bn)
    gg = run_case(nimg, 33, 65, 256, 512, True, use_bn)
    d = (e - gg).abs().max().item()
    print(f"nimg {nimg} bn {use_bn}: eager vs graph max diff {d:.3e} (max |dW| {e.abs().max().item():.3e})", flush=True)
