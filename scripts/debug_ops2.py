import sys; sys.path.insert(0, ".")
import maxsquareloss_amd
import torch, torch.nn.functional as F
torch.manual_seed(0)
def rel(a, b): return ((a.double().cpu() - b).abs().max() / b.abs().max()).item()
def case(name, x, w, stride=1, pad=0):
    gy_shape = F.conv2d(x, w, stride=stride, padding=pad).shape
    gy = torch.randn(gy_shape)
    xr, wr = x.double().requires_grad_(), w.double().requires_grad_()
    F.conv2d(xr, wr, stride=stride, padding=pad).backward(gy.double())
    xg, wg = x.cuda().requires_grad_(), w.cuda().requires_grad_()
    F.conv2d(xg, wg, stride=stride, padding=pad).backward(gy.cuda())
    xc, wc = x.clone().requires_grad_(), w.clone().requires_grad_()
    F.conv2d(xc, wc, stride=stride, padding=pad).backward(gy)
    print(name, "gpu dx", rel(xg.grad, xr.grad), "gpu dw", rel(wg.grad, wr.grad), "| cpu dx", rel(xc.grad, xr.grad), "cpu dw", rel(wc.grad, wr.grad), flush=True)
case("stem7x7/2", torch.randn(1, 3, 512, 1024) * 50, torch.randn(64, 3, 7, 7) * 0.01, 2, 3)
case("1x1 256->64 @129x257", torch.randn(1, 256, 129, 257), torch.randn(64, 256, 1, 1) * 0.01)
case("1x1 64->256 @65x129", torch.randn(1, 64, 65, 129), torch.randn(256, 64, 1, 1) * 0.01)
case("1x1/2 256->512", torch.randn(1, 256, 129, 257), torch.randn(512, 256, 1, 1) * 0.01, 2)
case("1x1 1024->256", torch.randn(1, 1024, 65, 129), torch.randn(256, 1024, 1, 1) * 0.01)
