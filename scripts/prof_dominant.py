"""The bench's dominant kernel alone: the layer3 dilated conv forward (256->256, d=2) at the
1024x512 feature size (65x129), launched through the same op as the training step.  Profiled
with rocprofv3 (--kernel-trace --stats, then separate --pmc passes) by scripts/gpu_counters.sh.

    prof_dominant.py [N] [H W MATH]     e.g. 20 96 161 fp16 (BASELINE configs[4]: 1280x760, fp16 MFMA)

NIMG (env, default 2): images per call - the trainer runs the source and target images as one pair
([C][2][H][W]), so the bench's dominant op covers two images."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from maxsquareloss_amd import ops  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 50
H, W = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (65, 129)
if len(sys.argv) > 4:
    ops.set_conv_math(sys.argv[4])
g = torch.Generator(device="cuda").manual_seed(0)
nimg = int(os.environ.get("NIMG", "2"))
x = torch.randn((1, 256, nimg, H, W) if nimg > 1 else (1, 256, H, W), device="cuda", generator=g)
w = torch.randn(256, 256, 3, 3, device="cuda", generator=g) * 0.02
cache = ops.PackCache()
# f16x3: in the step the input's absmax partials come from the BN kernel that produced it, so the
# op launches no absmax pass; the same here (computed once, outside the profiled loop's op calls)
q = ops._parts(x)
if q is not None:
    ops._tag_absmax(x, q[0])
with torch.no_grad():
    for _ in range(n):
        y = ops.dconv3x3(x, w, 2, cache)
torch.cuda.synchronize()
print("launches", n, "checksum", float(y.double().sum()))
