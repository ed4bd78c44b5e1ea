"""cProfile of the bench step's host side (5 steps after warm-up) on the GPU box: where the
Python / autograd / ctypes enqueue time goes."""
import cProfile, io, os, pstats, sys
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
pr = cProfile.Profile()
pr.enable()
for _ in range(5):
    tr.uda_step(*b)
pr.disable()
torch.cuda.synchronize()
out = io.StringIO()
pstats.Stats(pr, stream=out).sort_stats("tottime").print_stats(30)
print(out.getvalue())
