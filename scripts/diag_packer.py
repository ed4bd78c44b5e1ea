"""Does ops.PackBatch batch the step's packs?  Runs a few eager UDA iterations at 1024x512 and
prints the batch launches and the per-iteration lazy pack count (PackCache.get repacks)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from maxsquareloss_amd import ops  # noqa: E402
from maxsquareloss_amd.tools.solve_gta5 import UDATrainer, build_parser  # noqa: E402
from maxsquareloss_amd.tools.train_source import init_args  # noqa: E402
from maxsquareloss_amd.utils.synthetic import synthetic_image, synthetic_labels  # noqa: E402

lazy = [0]
orig = ops.PackCache.get


def counting_get(self, weights, cin, cout, for_dgrad):
    if self.key[for_dgrad] != self.key_of(weights):
        lazy[0] += 1
    return orig(self, weights, cin, cout, for_dgrad)


ops.PackCache.get = counting_get
argv = ["--crop_size", "1024,512", "--target_crop_size", "1024,512", "--imagenet_pretrained", "False", "--save_dir", "", "--multi", "False",
        "--iter_max", "1000"]
args, _, _ = init_args(build_parser().parse_args(argv))
tr = UDATrainer(args, cuda=True)
xs, ys, xt = synthetic_image(512, 1024, 1).cuda(), synthetic_labels(512, 1024, 19, 1).cuda(), synthetic_image(512, 1024, 2).cuda()
for it in range(4):
    lazy[0] = 0
    tr.uda_step(xs, ys, xt)
    torch.cuda.synchronize()
    jobs = tr.packer._jobs()
    stale = sum(c.key[d] != c.key_of(c.meta[d][0]) for c, d in jobs)
    print(f"iteration {it}: lazy repacks {lazy[0]}, batch launches so far {tr.packer.launches}, jobs {len(jobs)}, "
          f"stale after step {stale}", flush=True)
