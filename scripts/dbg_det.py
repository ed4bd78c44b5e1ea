"""Determinism probe: each conv op form run repeatedly on the same inputs, outputs compared bitwise."""
import sys, os, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from maxsquareloss_amd import ops
torch.manual_seed(0)
dev = "cuda"
def rep(name, f, n=6):
    ref = f()
    bad = 0
    for _ in range(n):
        o = f()
        if not torch.equal(o, ref):
            bad += 1
            d = (o - ref).abs().max().item()
    print(f"{name:40s} nondeterministic {bad}/{n}" + (f" maxdiff {d:.3e}" if bad else ""), flush=True)
for nimg in (1, 2):
    for (cin, cout, h, w, d) in [(256, 256, 65, 129, 2), (64, 64, 129, 257, 1), (512, 512, 65, 129, 4), (128, 128, 65, 129, 1)]:
        x = torch.randn(1, cin, nimg, h, w, device=dev) if nimg > 1 else torch.randn(1, cin, h, w, device=dev)
        wt = torch.randn(cout, cin, 3, 3, device=dev) * 0.02
        c = ops.PackCache()
        rep(f"dconv {cin}->{cout} {h}x{w} d{d} n{nimg}", lambda: ops.dconv3x3(x, wt, d, c))
    for (cin, cout, h, w) in [(1024, 256, 65, 129), (256, 1024, 65, 129), (64, 256, 129, 257), (256, 64, 129, 257)]:
        x = torch.randn(1, cin, nimg, h, w, device=dev) if nimg > 1 else torch.randn(1, cin, h, w, device=dev)
        wt = torch.randn(cout, cin, 1, 1, device=dev) * 0.02
        c = ops.PackCache(pointwise=True)
        rep(f"pconv {cin}->{cout} {h}x{w} n{nimg}", lambda: ops.pconv(x, wt, c))
    x = torch.randn(1, 3, nimg, 512, 1024, device=dev) * 50 if nimg > 1 else torch.randn(1, 3, 512, 1024, device=dev) * 50
    wt = torch.randn(64, 3, 7, 7, device=dev) * 0.05
    c = ops.PackCache(pointwise=True)
    rep(f"stem n{nimg}", lambda: ops.stem_conv(x, wt, 2, 3, c))
