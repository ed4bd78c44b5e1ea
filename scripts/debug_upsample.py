import sys; sys.path.insert(0, ".")
import numpy as np, torch, torch.nn.functional as F
from maxsquareloss_amd import ops
print("cpu capability", torch.backends.cpu.get_cpu_capability(), "threads", torch.get_num_threads())
f = np.float32
def idx(o_n, i_n):
    sc = f(i_n-1)/f(o_n-1); real = (sc*np.arange(o_n, dtype=np.float32)).astype(np.float32)
    i0 = np.minimum(np.floor(real).astype(np.int64), i_n-1); lam = np.clip(real-i0.astype(np.float32), 0, 1).astype(np.float32)
    return i0, i0+(i0 < i_n-1), (f(1)-lam).astype(f), lam
def fm(a, b, c): return (a.astype(np.float64)*b.astype(np.float64)+c.astype(np.float64)).astype(np.float32)
for (c,hi,wi,ho,wo) in [(19,65,129,512,1024),(19,33,65,256,512),(3,5,7,11,13)]:
    g = torch.Generator().manual_seed(hi)
    x = torch.randn(1, c, hi, wi, generator=g) * 3
    yr = F.interpolate(x, size=(ho, wo), mode="bilinear", align_corners=True)[0].numpy()
    yg = ops.upsample_bilinear(x.cuda(), (ho, wo))[0].cpu().numpy()
    h0,h1,a0,a1 = idx(ho,hi); w0,w1,b0,b1 = idx(wo,wi)
    X = x[0].numpy(); A0=a0[None,:,None];A1=a1[None,:,None];B0=b0[None,None,:];B1=b1[None,None,:]
    x00=X[:,h0][:,:,w0]; x01=X[:,h0][:,:,w1]; x10=X[:,h1][:,:,w0]; x11=X[:,h1][:,:,w1]
    em = fm(fm(x00,B0,x01*B1), A0, fm(x10,B0,x11*B1)*A1)
    print((c,hi,wi,ho,wo), "gpu!=cpu", np.count_nonzero(yg!=yr), "emu!=cpu", np.count_nonzero(em!=yr), "gpu!=emu", np.count_nonzero(yg!=em))
    bad = np.argwhere(yg != em)[:3]
    for b in bad: print(b, yg[tuple(b)], em[tuple(b)], yr[tuple(b)])
