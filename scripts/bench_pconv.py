"""Per-shape timing: HIP pointwise conv (fwd/dgrad/wgrad) vs MIOpen (F.conv2d + autograd)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, torch.nn.functional as F
from maxsquareloss_amd import ops, hip

def t(fn, iters=20):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3

shapes = [(64, 64, 129, 257), (64, 256, 129, 257), (256, 64, 129, 257), (128, 512, 65, 129), (512, 128, 65, 129),
          (512, 256, 65, 129), (512, 1024, 65, 129), (256, 1024, 65, 129), (1024, 256, 65, 129),
          (1024, 512, 65, 129), (1024, 2048, 65, 129), (512, 2048, 65, 129), (2048, 512, 65, 129)]
lib = hip.load()
tot_h = tot_m = 0.0
for cin, cout, h, w in shapes:
    x = torch.randn(1, cin, h, w, device="cuda")
    wt = torch.randn(cout, cin, 1, 1, device="cuda") * 0.05
    gy = torch.randn(1, cout, h, w, device="cuda")
    cache = ops.PackCache(pointwise=True)
    p = h * w
    gf = 2.0 * cin * cout * p / 1e9
    # HIP
    y = ops.pconv(x, wt, cache)
    packed = cache.get([wt], cin, cout, 0)
    packed_d = cache.get([wt], cin, cout, 1)
    s = hip.stream_ptr()
    wsf = hip.workspace(lib.msl_pconv_fwd_workspace(cin, cout, p), x.device)
    wsd = hip.workspace(lib.msl_pconv_dgrad_workspace(cin, cout, p), x.device)
    wsw = hip.workspace(lib.msl_pconv_wgrad_workspace(cin, cout, p), x.device)
    dx = torch.empty_like(x); dw = torch.empty_like(wt)
    hf = t(lambda: lib.msl_pconv_fwd(x.data_ptr(), packed.data_ptr(), y.data_ptr(), cin, cout, p, hip.counters(x.device).data_ptr(), wsf.data_ptr(), wsf.numel(), s))
    hd = t(lambda: lib.msl_pconv_dgrad(gy.data_ptr(), packed_d.data_ptr(), dx.data_ptr(), cin, cout, p, hip.counters(x.device).data_ptr(), wsd.data_ptr(), wsd.numel(), s))
    hw = t(lambda: lib.msl_pconv_wgrad(x.data_ptr(), gy.data_ptr(), dw.data_ptr(), cin, cout, p, 0, wsw.data_ptr(), wsw.numel(), s))
    # MIOpen
    mf = t(lambda: F.conv2d(x, wt))
    md = t(lambda: torch.ops.aten.convolution_backward(gy, x, wt, None, (1, 1), (0, 0), (1, 1), False, (0, 0), 1, (True, False, False)))
    mw = t(lambda: torch.ops.aten.convolution_backward(gy, x, wt, None, (1, 1), (0, 0), (1, 1), False, (0, 0), 1, (False, True, False)))
    tot_h += hf + hd + hw; tot_m += mf + md + mw
    print(f"{cin:5d}->{cout:5d} P {p:6d} {gf:6.2f} GF | HIP fwd {hf:7.1f} dgrad {hd:7.1f} wgrad {hw:7.1f} us"
          f" | MIOpen fwd {mf:7.1f} dgrad {md:7.1f} wgrad {mw:7.1f} us", flush=True)
print(f"sum HIP {tot_h:.0f} us, MIOpen {tot_m:.0f} us")
