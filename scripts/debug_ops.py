import sys; sys.path.insert(0, ".")
import maxsquareloss_amd
import torch, torch.nn.functional as F
torch.manual_seed(0)
def rel(a, b): return ((a.double().cpu() - b).abs().max() / b.abs().max()).item()
x = torch.randn(1, 3, 256, 512) * 50
w = torch.randn(64, 3, 7, 7) * 0.01
print("stem 7x7/2", rel(F.conv2d(x.cuda(), w.cuda(), stride=2, padding=3), F.conv2d(x.double(), w.double(), stride=2, padding=3)))
x = torch.randn(1, 256, 65, 129); w = torch.randn(64, 256, 1, 1) * 0.01
print("1x1 256->64", rel(F.conv2d(x.cuda(), w.cuda()), F.conv2d(x.double(), w.double())))
x = torch.randn(1, 64, 65, 129); w = torch.randn(256, 64, 1, 1) * 0.01
print("1x1 64->256", rel(F.conv2d(x.cuda(), w.cuda()), F.conv2d(x.double(), w.double())))
x = torch.randn(1, 256, 65, 129); w = torch.randn(512, 256, 1, 1) * 0.01
print("1x1 /2 256->512", rel(F.conv2d(x.cuda(), w.cuda(), stride=2), F.conv2d(x.double(), w.double(), stride=2)))
x = torch.randn(1, 64, 129, 257) * 3 + 1
g, b = torch.ones(64), torch.zeros(64)
yr = F.batch_norm(x.double(), torch.zeros(64, dtype=torch.float64), torch.ones(64, dtype=torch.float64), g.double(), b.double(), True, 0.1, 1e-5)
print("bn train", rel(F.batch_norm(x.cuda(), torch.zeros(64).cuda(), torch.ones(64).cuda(), g.cuda(), b.cuda(), True, 0.1, 1e-5), yr))
x = torch.randn(1, 64, 256, 512)
print("maxpool", rel(F.max_pool2d(x.cuda(), 3, 2, 1, ceil_mode=True), F.max_pool2d(x.double(), 3, 2, 1, ceil_mode=True)))
print("flags", torch.backends.cudnn.allow_tf32, torch.backends.cuda.matmul.allow_tf32, torch.backends.cudnn.enabled)
