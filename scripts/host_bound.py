"""Is the bench step host-bound?  Host enqueue time per uda_step (no sync inside the step) vs the
wall time per step once the GPU drains, at the bench's default workload."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from maxsquareloss_amd.tools.solve_gta5 import UDATrainer, build_parser
from maxsquareloss_amd.tools.train_source import init_args
from maxsquareloss_amd.utils.synthetic import synthetic_image, synthetic_labels

argv = ["--crop_size", "1024,512", "--target_crop_size", "1024,512", "--imagenet_pretrained", "False",
        "--save_dir", "", "--target_mode", "maxsquare", "--multi", "False", "--lambda_target", "0.1",
        "--iter_max", "200000"]
args, _, _ = init_args(build_parser().parse_args(argv))
tr = UDATrainer(args, cuda=True)
b = (synthetic_image(512, 1024, 0).cuda(), synthetic_labels(512, 1024, 19, 0).cuda(), synthetic_image(512, 1024, 500).cuda())
for _ in range(3):
    tr.uda_step(*b)
torch.cuda.synchronize()
N = 10
host = []
t0 = time.perf_counter()
for _ in range(N):
    h0 = time.perf_counter()
    tr.uda_step(*b)
    host.append(time.perf_counter() - h0)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print("per-step host enqueue (ms):", " ".join(f"{h*1e3:.1f}" for h in host))
torch.cuda.synchronize()
first = []
for _ in range(3):  # one step from a drained queue: the host cost alone
    torch.cuda.synchronize()
    h0 = time.perf_counter()
    tr.uda_step(*b)
    first.append(time.perf_counter() - h0)
torch.cuda.synchronize()
print("from a drained queue (ms):", " ".join(f"{h*1e3:.1f}" for h in first))
print(f"host enqueue per step: median {sorted(host)[N//2]*1e3:.2f} ms  (all {N}: {(t1-t0)/N*1e3:.2f} ms/step)"
      f"  wall incl. drain {(t2-t0)/N*1e3:.2f} ms/step  tail drain {(t2-t1)*1e3:.1f} ms")
