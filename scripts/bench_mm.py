"""1x1-conv GEMMs through torch.mm (rocBLAS vs hipBLASLt backends) vs MIOpen's conv path."""
import torch, torch.nn.functional as F

def t(fn, iters=20):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3

torch.backends.cuda.matmul.allow_tf32 = False
shapes = [(64, 256, 33153), (256, 64, 33153), (512, 128, 8385), (128, 512, 8385), (1024, 256, 8385), (256, 1024, 8385),
          (2048, 512, 8385), (512, 2048, 8385), (1024, 2048, 8385)]
for lib in ["rocblas", "hipblaslt"]:
    try:
        torch.backends.cuda.preferred_blas_library(lib)
    except Exception as e:
        print("cannot select", lib, e); continue
    tot = 0.0
    for cin, cout, p in shapes:
        x = torch.randn(cin, p, device="cuda"); w = torch.randn(cout, cin, device="cuda"); gy = torch.randn(cout, p, device="cuda")
        gf = 2 * cin * cout * p / 1e9
        f = t(lambda: torch.mm(w, x)); d = t(lambda: torch.mm(w.t(), gy)); wg = t(lambda: torch.mm(gy, x.t()))
        tot += f + d + wg
        print(f"{lib:9s} {cin:5d}->{cout:5d} P {p:6d}: fwd {f:7.1f} ({gf/f*1e3:5.1f} TF) dgrad {d:7.1f} ({gf/d*1e3:5.1f}) wgrad {wg:7.1f} ({gf/wg*1e3:5.1f})", flush=True)
    print(lib, "sum", round(tot))
tot = 0.0
for cin, cout, p in shapes:
    x = torch.randn(1, cin, 1, p, device="cuda"); w = torch.randn(cout, cin, 1, 1, device="cuda"); gy = torch.randn(1, cout, 1, p, device="cuda")
    f = t(lambda: F.conv2d(x, w))
    d = t(lambda: torch.ops.aten.convolution_backward(gy, x, w, None, (1, 1), (0, 0), (1, 1), False, (0, 0), 1, (True, False, False)))
    wg = t(lambda: torch.ops.aten.convolution_backward(gy, x, w, None, (1, 1), (0, 0), (1, 1), False, (0, 0), 1, (False, True, False)))
    tot += f + d + wg
    print(f"miopen    {cin:5d}->{cout:5d} P {p:6d}: fwd {f:7.1f} dgrad {d:7.1f} wgrad {wg:7.1f}", flush=True)
print("miopen sum", round(tot))
