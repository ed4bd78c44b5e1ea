"""Same-box A/B of the conv -> BN fusion (ops.FOLD) on the step's layer3 / layer4 shapes over an image pair:
forward = conv GEMM + BN (pieces summed by the BN kernel vs by k_sk_reduce), backward = data-gradient
GEMM + the producing BN's backward.  HIP events around R repetitions of each, median of 5 rounds.

    python scripts/bench_fold.py [R]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

from maxsquareloss_amd import ops  # noqa: E402

R = int(sys.argv[1]) if len(sys.argv) > 1 else 20
DEV = "cuda"


def chain(kind, cin, cout, h, w, d, res):
    g = torch.Generator().manual_seed(1)
    x = torch.relu(torch.randn(1, cin, 2, h, w, generator=g)).to(DEV).requires_grad_()
    k = 3 if kind == "3x3" else 1
    wt = (torch.randn(cout, cin, k, k, generator=g) * (0.5 / (cin * k * k) ** 0.5)).to(DEV).requires_grad_()
    r = torch.randn(1, cout, 2, h, w, generator=g).to(DEV) if res else None
    gy = torch.randn(1, cout, 2, h, w, generator=g).to(DEV)
    bn0, bn = nn.BatchNorm2d(cin).to(DEV).train(), nn.BatchNorm2d(cout).to(DEV).train()
    cache = ops.PackCache(pointwise=kind != "3x3")

    def run(fold):
        x.grad = wt.grad = None
        xin = ops.bn_act(bn0, x, relu=True)
        y = ops.dconv3x3(xin, wt, d, cache, fold) if kind == "3x3" else ops.pconv(xin, wt, cache, None, fold)
        out = ops.bn_act(bn, y, residual=r, relu=True)
        out.backward(gy)
    return run


def timeit(fn):
    """GPU time of fn (captured once as a hipGraph and replayed R times: no host launch gaps)."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(R):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / R * 1e3)
    return sorted(ts)[2]


for spec in [("1x1", 1024, 256, 65, 129, 0, False), ("3x3", 256, 256, 65, 129, 2, False),
             ("1x1", 256, 1024, 65, 129, 0, True), ("1x1", 2048, 512, 65, 129, 0, False),
             ("1x1", 512, 2048, 65, 129, 0, True)]:
    run = chain(*spec)
    t0 = timeit(lambda: run(0))
    t1 = timeit(lambda: run(3))
    print(f"{spec}: unfused {t0:8.1f} us  folded {t1:8.1f} us  (bn0 fwd/bwd + conv fwd/dgrad/wgrad + bn fwd/bwd)",
          flush=True)
