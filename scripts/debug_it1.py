"""Debug: after one UDA step + oracle re-sync, compare the it1 target forward (iwmulti config)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch, torch.nn.functional as F
from oracle import msl_oracle as orc
from maxsquareloss_amd.tools.solve_gta5 import UDATrainer, build_parser
from maxsquareloss_amd.tools.train_source import init_args
from maxsquareloss_amd.utils.synthetic import synthetic_image, synthetic_labels
H, W = 256, 512
argv = ["--crop_size", f"{W},{H}", "--target_crop_size", f"{W},{H}", "--imagenet_pretrained", "False",
        "--save_dir", "", "--num_classes", "19", "--target_mode", "IW_maxsquare", "--multi", "True",
        "--lambda_target", sys.argv[1] if len(sys.argv) > 1 else "0.09"]
args, _, _ = init_args(build_parser().parse_args(argv))
tr = UDATrainer(args, cuda=True); tr.args.iter_max = 200000
tr.optimizer.zero_grad()
xs, ys = synthetic_image(H, W, 0), synthetic_labels(H, W, 19, 0)
xt = synthetic_image(H, W, 500)
tr.uda_step(xs.cuda(), ys.cuda(), xt.cuda()); torch.cuda.synchronize()
sd = {k: v.detach().cpu().clone() for k, v in tr.model.state_dict().items()}
model = orc.Model(sd)
xt1 = synthetic_image(H, W, 501)
with torch.no_grad():
    tr.model.train()
    g2, g1 = tr.model(xt1.cuda())
    r2, r1 = orc.forward(model.params, model.buffers, xt1)
def nw(a, b): a, b = a.double().cpu(), b.double().cpu(); return ((a-b).norm()/b.norm()).item()
print("normwise x2", nw(g2, r2), "x1", nw(g1, r1))
for name, (g, r) in {"x2": (g2, r2), "x1": (g1, r1)}.items():
    print(name, "maxabs", (g.cpu()-r).abs().max().item(), "absmax ref", r.abs().max().item())
Pg, P2g = F.softmax(g2.cpu(), 1), F.softmax(g1.cpu(), 1)
Pr, P2r = F.softmax(r2, 1), F.softmax(r1, 1)
lg = orc.multi_guidance_label(Pg, P2g, 0.95); lr_ = orc.multi_guidance_label(Pr, P2r, 0.95)
print("mask gpu", (lg >= 0).sum().item(), "ref", (lr_ >= 0).sum().item(), "label diff", (lg != lr_).sum().item())
print("ce gpu", orc.ce(g1.cpu(), lg).item(), "ce ref", orc.ce(r1, lr_).item(), "ce gpu-logits ref-label", orc.ce(g1.cpu(), lr_).item())
mp = torch.maximum(Pr.max(1)[0], P2r.max(1)[0])
print("ref pixels with max p in [0.9499,0.9501]:", ((mp > 0.9499) & (mp < 0.9501)).sum().item())
# per-layer: features
# the test's path: a full step at it1 on both sides
cfg = dict(lr=2.5e-4, iter_max=200000, lambda_seg=0.1, IW_ratio=0.2, threshold=0.95,
           target_mode=tr.args.target_mode, multi=tr.args.multi, lambda_target=tr.args.lambda_target)
print("lambda_seg", tr.args.lambda_seg, "lambda_target", tr.args.lambda_target, "threshold", tr.threshold)
opt = orc.SGDMult(model.params, model.names, cfg["lr"])
for n, p in tr.model.named_parameters():
    st = tr.optimizer.state.get(p)
    if st is not None and n in opt.buf:
        opt.buf[n] = st["momentum_buffer"].detach().cpu().clone()
xs1, ys1 = synthetic_image(H, W, 1), synthetic_labels(H, W, 19, 1)
tr.uda_step(xs1.cuda(), ys1.cuda(), xt1.cuda()); torch.cuda.synchronize()
out = orc.uda_step(model, opt, xs1, ys1, xt1, cfg, 1)
print("step it1 gpu", tr.loss_val.item(), tr.loss_target.item(), tr.loss_target_2.item())
print("step it1 orc", out["loss_seg"], out["loss_target"], out["loss_target_2"])
