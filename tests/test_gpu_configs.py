"""Every BASELINE.json config at its real size, one UDA iteration against the CPU oracle (GPU only).

BASELINE.json configs, bs=1, counter-generated init, synthetic images:
  configs[1]  GTA5->CS MaxSquare, 1024x512, multi False, lambda_t 0.1       (tools/solve_gta5.py:335-387)
  configs[2]  the same step with IW-MaxSquare (the data-parallel config; one rank's step here)
  configs[3]  IW-MaxSquare + multi-level guidance, 1280x640, lambda_t 0.09  (solve_gta5.py:178-218)
  configs[4]  SYNTHIA->CS, 16 classes, 1280x760, IW + multi, every conv on the fp16 MFMA path
(configs[0], train_source at 512x256, is tests/test_gpu_parity.py::test_source_step_cfg0_matches_goldens.)

Bars:
  - fp32 configs (one iteration): the source CE and the target loss within 1e-3 relative of the fp32
    oracle; the guidance CE within 1e-3 plus the slack of the pixels that sit within rounding of its
    threshold / argmax decisions (test_gpu_model._guidance_slack); the IW class histogram within
    0.1 % of the pixels (argmax flips of random-init logits with near-equal classes, Q11); the SGD
    update per tensor within 3x the fp32 oracle's own distance to an fp64 oracle (the bs=1 network
    amplifies fp32 rounding through ~100 BN layers: the stem's weight gradient moves by a few % between
    two fp32 summation orders - tests/test_gpu_model.py), and the whole update within 2x in norm;
  - configs[4] (fp16 operands, fp32 sums; "parity is loss curve vs fp32 CPU within tolerance",
    SURVEY.md §8d): two iterations, each loss within 1e-2 of the fp32 oracle at iteration 0 and
    3e-2 at iteration 1 (the oracle re-synced to the GPU's weights in between, so the bar measures
    one iteration's fp16 rounding; the IW histogram and the update are not held: fp16 operand
    rounding (2^-11) moves 0.4 % of the random-init argmaxes and, amplified by the bs=1 BN layers,
    the early layers' gradients).
The measured values are printed (pytest -s / -rA) so the margins are visible in the log.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from oracle import msl_oracle as orc  # noqa: E402
from maxsquareloss_amd import ops  # noqa: E402
from maxsquareloss_amd.tools.solve_gta5 import UDATrainer, build_parser  # noqa: E402
from maxsquareloss_amd.tools.train_source import init_args  # noqa: E402
from maxsquareloss_amd.utils.synthetic import synthetic_image, synthetic_labels  # noqa: E402

CONFIGS = {
    "cfg1_maxsquare_1024x512": dict(w=1024, h=512, C=19, mode="maxsquare", multi=False, lt=0.1, math="fp32"),
    "cfg2_iw_1024x512": dict(w=1024, h=512, C=19, mode="IW_maxsquare", multi=False, lt=0.1, math="fp32"),
    "cfg3_iw_multi_1280x640": dict(w=1280, h=640, C=19, mode="IW_maxsquare", multi=True, lt=0.09, math="fp32"),
    "cfg4_synthia16_1280x760_fp16": dict(w=1280, h=760, C=16, mode="IW_maxsquare", multi=True, lt=0.1,
                                         math="fp16"),
}


def _resync(tr, model, opt):
    with torch.no_grad():
        for n, p in tr.model.named_parameters():
            model.params[n].copy_(p.detach().cpu())
        for n, b in tr.model.named_buffers():
            model.buffers[n].copy_(b.detach().cpu())
    for n, p in tr.model.named_parameters():
        st = tr.optimizer.state.get(p)
        if st is not None:
            opt.buf[n] = st["momentum_buffer"].detach().cpu().clone()


@pytest.mark.parametrize("name", list(CONFIGS))
def test_config_full_size(name):
    from test_gpu_model import _guidance_slack
    c = CONFIGS[name]
    h, w, C = c["h"], c["w"], c["C"]
    fp16 = c["math"] == "fp16"
    argv = ["--crop_size", f"{w},{h}", "--target_crop_size", f"{w},{h}", "--imagenet_pretrained", "False",
            "--save_dir", "", "--num_classes", str(C), "--target_mode", c["mode"], "--multi", str(c["multi"]),
            "--lambda_target", str(c["lt"]), "--conv_math", c["math"], "--iter_max", "200000"]
    args, _, _ = init_args(build_parser().parse_args(argv))
    tr = UDATrainer(args, cuda=True)
    try:
        cfg = dict(lr=args.lr, iter_max=200000, lambda_seg=args.lambda_seg, IW_ratio=args.IW_ratio,
                   threshold=args.threshold, target_mode=c["mode"], multi=args.multi, lambda_target=c["lt"])
        sd0 = {k: v.cpu().clone() for k, v in tr.model.state_dict().items()}
        model = orc.Model(sd0, C)
        opt = orc.SGDMult(model.params, model.names, cfg["lr"])
        m64 = None if fp16 else orc.Model(sd0, C, dtype=torch.float64)
        opt64 = None if fp16 else orc.SGDMult(m64.params, m64.names, cfg["lr"])
        tr.optimizer.zero_grad()
        for it in range(2 if fp16 else 1):
            if it:
                _resync(tr, model, opt)
            p0 = {n: p.detach().cpu().clone() for n, p in tr.model.named_parameters()}
            xs, ys = synthetic_image(h, w, 7 + it), synthetic_labels(h, w, C, 7 + it)
            xt = synthetic_image(h, w, 507 + it)
            tr.uda_step(xs.cuda(), ys.cuda(), xt.cuda())
            torch.cuda.synchronize()
            slack = (_guidance_slack(model, xt, cfg["threshold"], cfg["lambda_seg"] * c["lt"]) if args.multi else 0.0)
            out = orc.uda_step(model, opt, xs, ys, xt, cfg, it)
            if m64 is not None:
                orc.uda_step(m64, opt64, xs, ys, xt, cfg, it)
            tol = (1e-2 if it == 0 else 3e-2) if fp16 else 1e-3
            mine = {"loss_seg": tr.loss_val.item(), "loss_target": tr.loss_target.item()}
            if args.multi:
                mine["loss_target_2"] = tr.loss_target_2.item()
            for k, v in mine.items():
                rel = abs(v - out[k]) / max(abs(out[k]), 1e-30)
                print(f"{name} it{it} {k}: gpu {v:.7g} oracle {out[k]:.7g} rel {rel:.2e} (slack {slack:.2e})")
                ab = slack if k == "loss_target_2" else 0.0
                assert v == pytest.approx(out[k], rel=tol, abs=ab), (name, it, k, v, out[k])
            if c["mode"] == "IW_maxsquare":
                hg = tr.target_loss.last_hist.cpu().numpy().astype(np.int64)
                flips = int(np.abs(hg - out["hist"]).sum()) // 2
                print(f"{name} it{it} IW histogram: {flips} argmax flips of {h * w} pixels")
                assert hg.sum() == out["hist"].sum() == h * w
                if not fp16:
                    assert flips <= 0.001 * h * w, (name, hg, out["hist"])
            if m64 is None:
                continue
            e_gpu_all = e_cpu_all = 0.0
            worst = (0.0, None)
            for n, p in tr.model.named_parameters():
                if not p.requires_grad:
                    continue
                du = p.detach().cpu().double() - p0[n].double()
                dr = model.params[n].detach().double() - p0[n].double()
                d64 = m64.params[n].detach() - p0[n].double()
                if d64.abs().max() == 0:
                    assert du.abs().max() == 0 and dr.abs().max() == 0, n  # dead parameters (Q1) untouched
                    continue
                e_gpu, e_cpu = (du - d64).norm().item(), (dr - d64).norm().item()
                e_gpu_all += e_gpu ** 2
                e_cpu_all += e_cpu ** 2
                ratio = e_gpu / max(e_cpu, 1e-3 * d64.norm().item())
                if ratio > worst[0]:
                    worst = (ratio, n)
                assert e_gpu <= max(3 * e_cpu, 1e-3 * d64.norm().item()), (name, n, e_gpu, e_cpu)
            print(f"{name} SGD update vs fp64: gpu {e_gpu_all ** 0.5:.3e} cpu-fp32 {e_cpu_all ** 0.5:.3e} "
                  f"(worst tensor ratio {worst[0]:.2f} at {worst[1]})")
            assert e_gpu_all <= 4 * e_cpu_all, (name, e_gpu_all ** 0.5, e_cpu_all ** 0.5)
    finally:
        ops.set_conv_math("fp32")


def test_config5_fp16_loss_curve():
    """configs[4]'s parity criterion, "loss curve vs fp32 CPU within tolerance" (SURVEY.md §8d), at a
    reduced 16-class size (640x380, the same 16-class heads, IW + multi, every conv on the fp16 MFMA
    path; tools/solve_gta5.py:335-387):
      - ten iterations with the fp32 oracle re-synced to the GPU state before each one: every
        iteration's losses within 1e-2 of the oracle's (one iteration's fp16 operand rounding), the
        guidance CE with its threshold slack on top, the IW histogram within 2 % of the pixels;
      - then five iterations WITHOUT re-syncing (both sides from the same state): the curve's drift
        printed per iteration and held within 2e-1 relative - fp16 rounding compounds through the
        updates of a random-init bs=1 network, and the IW argmax weights and the guidance threshold
        make the free trajectory chaotic: two stream-K partitions of the same fp16 GEMMs (r04) drifted
        1.7e-2 and 8.9e-2 on loss_target_2 by the fifth free iteration; no divergence."""
    from test_gpu_model import _guidance_slack
    h, w, C = 380, 640, 16
    argv = ["--crop_size", f"{w},{h}", "--target_crop_size", f"{w},{h}", "--imagenet_pretrained", "False",
            "--save_dir", "", "--num_classes", str(C), "--target_mode", "IW_maxsquare", "--multi", "True",
            "--lambda_target", "0.1", "--conv_math", "fp16", "--iter_max", "200000"]
    args, _, _ = init_args(build_parser().parse_args(argv))
    tr = UDATrainer(args, cuda=True)
    try:
        cfg = dict(lr=args.lr, iter_max=200000, lambda_seg=args.lambda_seg, IW_ratio=args.IW_ratio,
                   threshold=args.threshold, target_mode="IW_maxsquare", multi=True, lambda_target=0.1)
        model = orc.Model({k: v.cpu().clone() for k, v in tr.model.state_dict().items()}, C)
        opt = orc.SGDMult(model.params, model.names, cfg["lr"])
        tr.optimizer.zero_grad()
        keys = ("loss_seg", "loss_target", "loss_target_2")
        for it in range(15):
            resync = it < 10
            if resync:
                _resync(tr, model, opt)
            xs, ys = synthetic_image(h, w, 40 + it), synthetic_labels(h, w, C, 40 + it)
            xt = synthetic_image(h, w, 540 + it)
            tr.uda_step(xs.cuda(), ys.cuda(), xt.cuda())
            torch.cuda.synchronize()
            slack = _guidance_slack(model, xt, cfg["threshold"], cfg["lambda_seg"] * cfg["lambda_target"])
            out = orc.uda_step(model, opt, xs, ys, xt, cfg, it)
            mine = dict(zip(keys, (tr.loss_val.item(), tr.loss_target.item(), tr.loss_target_2.item())))
            hg = tr.target_loss.last_hist.cpu().numpy().astype(np.int64)
            flips = int(np.abs(hg - out["hist"]).sum()) // 2
            rels = {k: abs(mine[k] - out[k]) / max(abs(out[k]), 1e-30) for k in keys}
            print(f"cfg5 fp16 it{it} {'resynced' if resync else 'free'}: " +
                  " ".join(f"{k} {mine[k]:.6g}/{out[k]:.6g} ({rels[k]:.1e})" for k in keys) +
                  f" IW flips {flips} of {h * w} (guidance slack {slack:.1e})")
            tol = 1e-2 if resync else 2e-1
            for k in keys:
                ab = slack if k == "loss_target_2" else 0.0
                assert mine[k] == pytest.approx(out[k], rel=tol, abs=ab), (it, k, mine[k], out[k])
            if resync:
                assert flips <= 0.02 * h * w, (it, flips)
    finally:
        ops.set_conv_math("fp32")
