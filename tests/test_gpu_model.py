"""End-to-end parity of the MI355X training step against the oracle and the reference goldens.

Config 1 shapes (512x256, C=19), counter-initialised weights (seed 12345), the
same synthetic images as oracle/gen_golden.py.  Bar:
logits and losses within 1e-3 relative (normwise for tensors); IW class
histograms compared exactly where the logits agree (a few argmax flips are
inherent end to end - we allow <= 0.1% of pixels); parameters after two SGD
steps within 1e-4 relative per-tensor sums.
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from oracle import msl_oracle as orc  # noqa: E402
from maxsquareloss_amd.tools.solve_gta5 import UDATrainer, build_parser  # noqa: E402
from maxsquareloss_amd.tools.train_source import init_args  # noqa: E402
from maxsquareloss_amd.utils.synthetic import synthetic_image, synthetic_labels  # noqa: E402

GOLD = os.path.join(os.path.dirname(__file__), "golden")
H, W = 256, 512


def _args(extra):
    argv = ["--crop_size", f"{W},{H}", "--target_crop_size", f"{W},{H}", "--imagenet_pretrained", "False",
            "--save_dir", "", "--num_classes", "19"] + extra
    args, _, _ = init_args(build_parser().parse_args(argv))
    return args


def _normwise(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).abs().max() / b.abs().max()).item()


def test_forward_matches_oracle():
    tr = UDATrainer(_args(["--target_mode", "maxsquare", "--multi", "False"]), cuda=True)
    ref = orc.Model({k: v.cpu() for k, v in tr.model.state_dict().items()})
    x = synthetic_image(H, W, 0)
    with torch.no_grad():
        x2, x1 = tr.model(x.cuda())
        r2, r1 = ref(x)
    assert _normwise(x2, r2) < 1e-3
    assert _normwise(x1, r1) < 1e-3
    # BN running statistics updated identically (train mode, momentum 0.1, Q9)
    for k, v in tr.model.state_dict().items():
        if k.endswith("running_var") or k.endswith("running_mean"):
            assert _normwise(v, ref.buffers[k]) < 1e-3, k


@pytest.mark.parametrize("tag,extra", [
    ("ms", ["--target_mode", "maxsquare", "--multi", "False", "--lambda_target", "0.1"]),
    ("iwmulti", ["--target_mode", "IW_maxsquare", "--multi", "True", "--lambda_target", "0.09"])])
def test_uda_steps_match_goldens_and_oracle(tag, extra):
    g = np.load(os.path.join(GOLD, "step_cfg1.npz"), allow_pickle=False)
    tr = UDATrainer(_args(extra), cuda=True)
    tr.args.iter_max = 200000
    cfg = dict(lr=2.5e-4, iter_max=200000, lambda_seg=0.1, IW_ratio=0.2, threshold=0.95,
               target_mode=tr.args.target_mode, multi=tr.args.multi, lambda_target=tr.args.lambda_target)
    model = orc.Model({k: v.cpu() for k, v in tr.model.state_dict().items()})
    opt = orc.SGDMult(model.params, model.names, cfg["lr"])
    tr.optimizer.zero_grad()
    for it in range(2):
        xs, ys = synthetic_image(H, W, it), synthetic_labels(H, W, 19, it)
        xt = synthetic_image(H, W, 500 + it)
        tr.uda_step(xs.cuda(), ys.cuda(), xt.cuda())
        torch.cuda.synchronize()
        out = orc.uda_step(model, opt, xs, ys, xt, cfg, it)
        mine = {"loss_seg": tr.loss_val.item(), "loss_target": tr.loss_target.item()}
        if tr.args.multi:
            mine["loss_target_2"] = tr.loss_target_2.item()
        for k, v in mine.items():
            assert v == pytest.approx(out[k], rel=1e-3), f"{k} it{it} vs oracle"
            assert v == pytest.approx(float(g[f"{tag}_it{it}_{k}"]), rel=1e-3), f"{k} it{it} vs golden"
        if tr.args.target_mode == "IW_maxsquare":
            h = tr.target_loss.last_hist.cpu().numpy().astype(np.int64)
            assert np.abs(h - out["hist"]).sum() <= 2 * 0.001 * H * W
    names = [n for n, _ in tr.model.named_parameters()]
    mine = {n: p.detach().double().sum().item() for n, p in tr.model.named_parameters()}
    gsum = dict(zip(names, g[f"{tag}_param_sum"]))
    for n in names:
        ref = model.params[n].double().sum().item()
        scale = max(abs(ref), model.params[n].double().abs().sum().item() * 1e-3, 1e-6)
        assert abs(mine[n] - ref) / scale < 1e-3, n
        assert abs(mine[n] - gsum[n]) / scale < 1e-3, n
