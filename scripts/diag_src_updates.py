"""Diagnostic: per-tensor update of the configs[0] source step, GPU vs CPU fp32 oracle vs fp64 oracle."""
import argparse, sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from oracle import msl_oracle as orc
from maxsquareloss_amd.tools.train_source import Trainer, add_train_args, init_args
from maxsquareloss_amd.utils.synthetic import synthetic_image, synthetic_labels
H, W = 256, 512
args, _, _ = init_args(add_train_args(argparse.ArgumentParser()).parse_args(
    ["--crop_size", f"{W},{H}", "--imagenet_pretrained", "False", "--save_dir", "", "--iter_max", "200000"]))
tr = Trainer(args, cuda=True)
g = np.load("tests/golden/step_cfg1.npz")
sd0 = {k: v.cpu().clone() for k, v in tr.model.state_dict().items()}
m32, m64 = orc.Model(sd0), orc.Model(sd0, dtype=torch.float64)
o32, o64 = orc.SGDMult(m32.params, m32.names, 2.5e-4), orc.SGDMult(m64.params, m64.names, 2.5e-4)
cfg = dict(lr=2.5e-4, iter_max=200000, lambda_seg=0.1, multi=True)
p0 = {n: p.detach().cpu().double().clone() for n, p in tr.model.named_parameters()}
names = [n for n, _ in tr.model.named_parameters()]
for it in range(2):
    x, y = synthetic_image(H, W, 100 + it), synthetic_labels(H, W, 19, 100 + it)
    tr.poly_lr_scheduler(tr.optimizer, init_lr=2.5e-4, iter=it, max_iter=200000, power=0.9)
    l = tr.source_step(x.cuda(), y.cuda()).item()
    a = orc.source_step(m32, o32, x, y, cfg, it)["loss"]
    b = orc.source_step(m64, o64, x, y, cfg, it)["loss"]
    print(f"it{it} loss gpu {l:.7f} cpu32 {a:.7f} cpu64 {b:.7f} golden {float(g[f'src_it{it}_loss']):.7f}", flush=True)
    for n in names[:12] + ["layer3.5.conv2.weight", "layer4.2.conv3.weight", "layer6.conv2d_list.0.weight"]:
        du = dict(tr.model.named_parameters())[n].detach().cpu().double() - p0[n]
        d3 = m32.params[n].detach().double() - p0[n]
        d6 = m64.params[n].detach() - p0[n]
        print(f"  {n:34s} sum gpu {du.sum():+.5e} c32 {d3.sum():+.5e} c64 {d6.sum():+.5e} | norm gpu {du.norm():.4e} c64 {d6.norm():.4e} "
              f"| err gpu {(du-d6).norm()/max(d6.norm(),1e-30):.3e} c32 {(d3-d6).norm()/max(d6.norm(),1e-30):.3e}", flush=True)
ps = np.array([p.detach().double().sum().item() for p in tr.model.parameters()])
p3 = np.array([m32.params[n].double().sum().item() for n in names])
p6 = np.array([m64.params[n].double().sum().item() for n in names])
gs = g["src_param_sum"]
print("golden vs c32 max rel", np.max(np.abs(p3 - gs) / (np.abs(gs) + 1e-6)), "gpu", np.max(np.abs(ps - gs) / (np.abs(gs) + 1e-6)), "c64", np.max(np.abs(p6 - gs) / (np.abs(gs) + 1e-6)))
