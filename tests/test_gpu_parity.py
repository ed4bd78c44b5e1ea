"""The HIP path against the reference's own fixtures (GPU only).

tests/golden/*.npz were written by oracle/gen_golden.py from the reference's
deeplab_multi.py / loss.py (imported by path in the survey container) and its
SGD through torch.optim.SGD(foreach=False).  Here they are fed straight to the
HIP kernels, not only to the oracle:
  - loss_kat.npz: C = 19/16/13 logits, the argmax-tie case, the all-ignored CE
    -> the fused loss kernels: loss and d logits within 1e-5, IW histogram,
    argmax and multi-level guidance label bit-exact (utils/loss.py:69-119,
    solve_gta5.py:206-213);
  - conv_kat.npz: the reference's Bottleneck.conv2 (d=2, d=4) and
    Classifier_Module (ASPP, early return Q1) on counter-generated inputs ->
    msl_dconv_* through ops.dconv3x3 / ops.aspp2, both fp32 matrix-core forms;
  - step_cfg1.npz: configs[0], tools/train_source.py at 512x256 -> Trainer.source_step;
plus the IW histogram bit-exact given the oracle's own logits and a
10-iteration UDA loss curve against the oracle re-synced every iteration.
"""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from oracle import msl_oracle as orc  # noqa: E402
from maxsquareloss_amd import ops  # noqa: E402
from maxsquareloss_amd.utils.synthetic import counter_normal, init_weights, synthetic_image, synthetic_labels  # noqa: E402

GOLD = os.path.join(os.path.dirname(__file__), "golden")
DEV = "cuda"


def gold(name):
    return np.load(os.path.join(GOLD, name), allow_pickle=False)


def _rel(a, b):
    a = torch.as_tensor(a).detach().double().cpu()
    b = torch.as_tensor(b).detach().double().cpu()
    return (a - b).abs().max().item() / max(b.abs().max().item(), 1e-30)


@pytest.fixture(params=["mfma_f32", "bf16x6", "f16x3"])
def f32_form(request):
    prev = ops.set_f32_form(request.param)
    yield request.param
    ops.set_f32_form(prev)


# ----------------------------------------------------------------------------- losses on loss_kat
@pytest.mark.parametrize("C", [19, 16, 13])
def test_fused_losses_on_reference_kat(C):
    g = gold("loss_kat.npz")
    low = torch.from_numpy(g[f"C{C}_low"]).to(DEV)
    low2 = torch.from_numpy(g[f"C{C}_low2"]).to(DEV)
    y = torch.from_numpy(g[f"C{C}_y"]).to(DEV)
    hw = (64, 128)

    def run(fn):
        lg = low.clone().requires_grad_()
        out = fn(lg)
        loss = out[0] if isinstance(out, tuple) else out
        loss.backward()
        torch.cuda.synchronize()
        return out, lg.grad

    # MaxSquare (loss.py:104-119)
    out, d = run(lambda t: ops.maxsquare_up(t, hw))
    assert out.item() == pytest.approx(float(g[f"C{C}_ms"]), rel=1e-5)
    assert _rel(d, g[f"C{C}_ms_dlow"]) < 1e-5
    # IW MaxSquare (loss.py:69-102): histogram and argmax bit-exact
    (out, hist, _w), d = run(lambda t: ops.iw_maxsquare_up(t, hw, 0.2))
    assert np.array_equal(hist.cpu().numpy().astype(np.int64), g[f"C{C}_iw_hist"]), "IW histogram"
    assert out.item() == pytest.approx(float(g[f"C{C}_iw"]), rel=1e-5)
    assert _rel(d, g[f"C{C}_iw_dlow"]) < 1e-5
    arg, _ = ops.loss_labels_up(low, None, hw)
    assert np.array_equal(arg.cpu().numpy().reshape(g[f"C{C}_argmax"].shape), g[f"C{C}_argmax"].astype(np.int32))
    # CE(ignore=-1) (train_source.py:128)
    out, d = run(lambda t: ops.ce_up(t, y.reshape(-1), hw))
    assert out.item() == pytest.approx(float(g[f"C{C}_ce"]), rel=1e-5)
    assert _rel(d, g[f"C{C}_ce_dlow"]) < 1e-5
    # multi-level guidance at the default and a permissive threshold: label bit-exact
    for thr in (0.95, 0.5):
        t = str(thr).replace(".", "p")
        _, lab = ops.loss_labels_up(low, low2, hw, thr)
        want = g[f"C{C}_multi{t}_label"].astype(np.int32)
        assert np.array_equal(lab.cpu().numpy().reshape(want.shape), want), f"multi label thr {thr}"
        ref = float(g[f"C{C}_multi{t}_ce"])
        lg = low.clone().requires_grad_()
        out = ops.multi_ce_up(lg, low2, hw, thr)
        if np.isnan(ref):
            assert np.isnan(out.item())
            continue
        out.backward()
        torch.cuda.synchronize()
        assert out.item() == pytest.approx(ref, rel=1e-5)
        assert _rel(lg.grad, g[f"C{C}_multi{t}_dlow"]) < 1e-5


def test_argmax_ties_and_all_ignored_on_reference_kat():
    g = gold("loss_kat.npz")
    tie = torch.from_numpy(g["tie_logits"]).to(DEV)  # exact ties between classes 3 and 7; pixel 0 all equal
    hw = tuple(tie.shape[2:])  # identity interpolation: the loss sees the logits themselves
    arg, _ = ops.loss_labels_up(tie, None, hw)
    assert np.array_equal(arg.cpu().numpy().reshape(g["tie_argmax"].shape), g["tie_argmax"].astype(np.int32)), \
        "first-max argmax on exact ties"
    out, hist, _ = ops.iw_maxsquare_up(tie, hw, 0.2)
    assert out.item() == pytest.approx(float(g["tie_iw"]), rel=1e-5)
    want = np.bincount(g["tie_argmax"].reshape(-1), minlength=19)
    assert np.array_equal(hist.cpu().numpy(), want)
    # all pixels ignored: nan loss (quirk Q8) and a zero gradient
    low = torch.zeros(1, 19, 4, 8, device=DEV, requires_grad=True)
    out = ops.ce_up(low, torch.full((32,), -1, dtype=torch.int64, device=DEV), (4, 8))
    assert np.isnan(out.item()) and np.isnan(float(g["allignored_ce"]))
    out.backward()
    assert torch.count_nonzero(low.grad).item() == 0


def test_iw_histogram_bit_exact_on_oracle_logits():
    """class histograms bit-exact given identical logits.  The oracle's own low-res
    x2 logits (torch-CPU forward of the random-init model at 512x256) go to the HIP IW loss;
    its histogram must equal the oracle's histc of argmax(softmax(upsample)) exactly."""
    from maxsquareloss_amd.graphs.models.deeplab_multi import DeeplabMulti
    h, w = 256, 512
    m = init_weights(DeeplabMulti(19, pretrained=False), 12345)
    model = orc.Model(m.state_dict())
    x = synthetic_image(h, w, 500)
    with torch.no_grad():
        x2_low, x1_low = orc.forward_low(model.params, model.buffers, x)
        P = F.softmax(F.interpolate(x2_low, size=(h, w), mode="bilinear", align_corners=True), 1)
        hist_ref, _, arg_ref = orc.iw_hist_weights(P, 0.2, 19)
    out, hist, _ = ops.iw_maxsquare_up(x2_low.to(DEV).contiguous(), (h, w), 0.2)
    assert np.array_equal(hist.cpu().numpy().astype(np.int64), hist_ref.numpy().astype(np.int64))
    arg, _ = ops.loss_labels_up(x2_low.to(DEV).contiguous(), None, (h, w))
    assert torch.equal(arg.cpu().long(), arg_ref.reshape(-1))
    with torch.no_grad():
        lt, _ = orc.iw_maxsquare(P, 0.2, 19)
    assert out.item() == pytest.approx(lt.item(), rel=1e-5)


# ----------------------------------------------------------------------------- convs on conv_kat
def _chk(t, g, prefix, rtol=1e-5):
    a = t.detach().double().cpu().numpy()
    flat = a.reshape(-1)
    scale = np.abs(flat).max()
    np.testing.assert_allclose(flat[g[prefix + "_idx"]], g[prefix + "_sample"], rtol=rtol, atol=rtol * scale)
    # per-channel sums (dim 0 of the reference tensor's natural layout) and the grand sum
    ch = a.reshape(a.shape[0] if a.shape[0] > 1 else a.shape[1], -1).sum(1)
    np.testing.assert_allclose(ch, g[prefix + "_chsum"], rtol=rtol, atol=rtol * float(g[prefix + "_abssum"]) / ch.size ** 0.5)
    assert a.sum() == pytest.approx(float(g[prefix + "_sum"]), rel=rtol, abs=rtol * float(g[prefix + "_abssum"]))


def test_dilated_convs_on_reference_kat(f32_form):
    """Bottleneck.conv2 of the reference (deeplab_multi.py:17-18) at layer3 (d=2, 256 ch) and layer4
    (d=4, 512 ch): forward, data gradient and weight gradient of the HIP kernels vs its outputs."""
    g = gold("conv_kat.npz")
    for name in ("d2", "d4"):
        planes, h, w, dil = (int(v) for v in g[f"{name}_meta"])
        wt = torch.from_numpy(counter_normal(5, f"conv_{name}_w", planes * planes * 9, 0.01)).view(planes, planes, 3, 3)
        x = torch.from_numpy(counter_normal(6, f"conv_{name}_x", planes * h * w)).view(1, planes, h, w)
        gy = torch.from_numpy(counter_normal(7, f"conv_{name}_gy", planes * h * w)).view(1, planes, h, w)
        xg, wg = x.to(DEV).requires_grad_(), wt.to(DEV).requires_grad_()
        y = ops.dconv3x3(xg, wg, dil, ops.PackCache())
        y.backward(gy.to(DEV))
        torch.cuda.synchronize()
        _chk(y, g, f"{name}_y")
        _chk(xg.grad, g, f"{name}_dx")
        _chk(wg.grad, g, f"{name}_dw")


def test_aspp_on_reference_kat(f32_form):
    """Classifier_Module (deeplab_multi.py:51-66) with its early return (Q1): branches 0 and 1 only."""
    g = gold("conv_kat.npz")
    h, w = 17, 33
    for head, cin in (("aspp5", 1024), ("aspp6", 2048)):
        ws = [torch.from_numpy(counter_normal(8, f"{head}_w{i}", 19 * cin * 9, 0.01)).view(19, cin, 3, 3) for i in range(2)]
        bs = [torch.from_numpy(counter_normal(9, f"{head}_b{i}", 19, 0.01)) for i in range(2)]
        x = torch.from_numpy(counter_normal(10, f"{head}_x", cin * h * w)).view(1, cin, h, w)
        gy = torch.from_numpy(counter_normal(11, f"{head}_gy", 19 * h * w)).view(1, 19, h, w)
        dev = [t.to(DEV).requires_grad_() for t in (x, ws[0], bs[0], ws[1], bs[1])]
        y = ops.aspp2(dev[0], dev[1], dev[2], dev[3], dev[4], 6, 12, ops.PackCache())
        y.backward(gy.to(DEV))
        torch.cuda.synchronize()
        _chk(y, g, f"{head}_y")
        _chk(dev[0].grad, g, f"{head}_dx")
        for i in range(2):
            assert bool(g[f"{head}_w{i}_hasgrad"])
            _chk(dev[1 + 2 * i].grad, g, f"{head}_dw{i}")
            np.testing.assert_allclose(dev[2 + 2 * i].grad.cpu().numpy(), g[f"{head}_db{i}"], rtol=1e-5,
                                       atol=1e-5 * np.abs(g[f"{head}_db{i}"]).max())
        assert not bool(g[f"{head}_w2_hasgrad"]) and not bool(g[f"{head}_w3_hasgrad"])


# ----------------------------------------------------------------------------- configs[0]: train_source
H, W = 256, 512


def _resync(tr, model, opt):
    """Copy the GPU trainer's parameters, BN buffers and momentum buffers into the oracle."""
    with torch.no_grad():
        for n, p in tr.model.named_parameters():
            model.params[n].copy_(p.detach().cpu())
        for n, b in tr.model.named_buffers():
            model.buffers[n].copy_(b.detach().cpu())
    for n, p in tr.model.named_parameters():
        st = tr.optimizer.state.get(p)
        if st is not None:
            opt.buf[n] = st["momentum_buffer"].detach().cpu().clone()


def _update_within_fp32_envelope(tr, p0, model, m64):
    """The SGD update per tensor: |GPU - fp64| <= 3x |CPU fp32 - fp64| (through ~100 bs=1 BN
    layers fp32 rounding is amplified; this is the reference arithmetic's own error)."""
    for n, p in tr.model.named_parameters():
        if not p.requires_grad:
            continue
        du = p.detach().cpu().double() - p0[n].double()
        dr = model.params[n].detach().double() - p0[n].double()
        d64 = m64.params[n].detach() - p0[n].double()
        if d64.abs().max() == 0:
            assert du.abs().max() == 0 and dr.abs().max() == 0, n
            continue
        e_gpu = (du - d64).norm().item()
        e_cpu = (dr - d64).norm().item()
        assert e_gpu <= max(3 * e_cpu, 1e-3 * d64.norm().item()), (n, e_gpu, e_cpu)


def test_source_step_cfg0_matches_goldens():
    """BASELINE configs[0]: tools/train_source.py (DeepLabv2-ResNet101, 512x256, CE(x2)+0.1 CE(x1),
    zero_grad -> backward -> step, train_source.py:233-264) for two iterations through
    Trainer.source_step, against the reference's src_it{0,1}_loss / src_param_sum goldens.

    The bs=1 random-init network is chaotic from the second iteration on: fp32 rounding of the
    first update (a few % of the stem's gradient) changes the second update by 30-90 % in every
    fp32 implementation (the CPU oracle vs an fp64 oracle on the same host, measured on the GPU
    box in r02 with a diagnostic script since deleted, commit b6a08cc), so the reference's own fp32 runs on two hosts disagree on
    src_param_sum by far more than rounding.  The bars are therefore:
      it0: loss within 1e-3 of the golden and the oracle; the update per tensor within 3x the fp32
           oracle's own distance to the fp64 oracle;
      it1: loss within 1e-3 of an oracle re-synced to the GPU state (rounding only); against the
           lock-step fp64 oracle, as aggregates over all tensors (per tensor the chaotic update
           lands anywhere in the envelope): the update within 2x the fp32 oracle's distance (in
           norm), the loss and the summed per-tensor parameter-sum errors within 3x the spread of
           the two fp32 CPU runs (this host's oracle and the golden's src_it1_loss /
           src_param_sum)."""
    from maxsquareloss_amd.tools.train_source import Trainer, add_train_args, init_args
    import argparse
    argv = ["--crop_size", f"{W},{H}", "--imagenet_pretrained", "False", "--save_dir", "", "--num_classes", "19",
            "--iter_max", "200000"]
    args, _, _ = init_args(add_train_args(argparse.ArgumentParser()).parse_args(argv))
    tr = Trainer(args, cuda=True)
    assert args.multi  # the fork's default (train_source.py:825-826, quirk Q7)
    g = gold("step_cfg1.npz")
    sd0 = {k: v.cpu().clone() for k, v in tr.model.state_dict().items()}
    model, m64 = orc.Model(sd0), orc.Model(sd0, dtype=torch.float64)
    opt, opt64 = orc.SGDMult(model.params, model.names, 2.5e-4), orc.SGDMult(m64.params, m64.names, 2.5e-4)
    cfg = dict(lr=2.5e-4, iter_max=200000, lambda_seg=0.1, multi=True)
    for it in range(2):
        x, y = synthetic_image(H, W, 100 + it), synthetic_labels(H, W, 19, 100 + it)
        p_before = {n: p.detach().cpu().clone() for n, p in tr.model.named_parameters()}
        if it == 1:  # an oracle that starts iteration 1 from exactly the GPU's state
            mr = orc.Model({k: v.cpu().clone() for k, v in tr.model.state_dict().items()})
            optr = orc.SGDMult(mr.params, mr.names, 2.5e-4)
            _resync(tr, mr, optr)
            lr_ = orc.source_step(mr, optr, x, y, cfg, it)["loss"]
        c_before = {n: model.params[n].detach().clone() for n in model.names}
        s_before = {n: m64.params[n].detach().clone() for n in m64.names}
        tr.poly_lr_scheduler(tr.optimizer, init_lr=2.5e-4, iter=it, max_iter=200000, power=0.9)
        loss = tr.source_step(x.to(DEV), y.to(DEV)).item()
        torch.cuda.synchronize()
        l32 = orc.source_step(model, opt, x, y, cfg, it)["loss"]
        l64 = orc.source_step(m64, opt64, x, y, cfg, it)["loss"]
        gl = float(g[f"src_it{it}_loss"])
        if it == 0:
            assert loss == pytest.approx(l32, rel=1e-3), "it0 vs oracle"
            assert loss == pytest.approx(gl, rel=1e-3), "it0 vs reference golden"
        else:
            assert loss == pytest.approx(lr_, rel=1e-3), "it1 vs the re-synced oracle"
            # two independent fp32 runs of the reference arithmetic: this host's oracle and the
            # golden's (another CPU): the GPU must sit within 3x their spread around fp64
            spread = max(abs(l32 - l64), abs(gl - l64))
            assert abs(loss - l64) <= 3 * spread + 1e-3 * abs(l64), ("it1 vs fp64", loss, l32, gl, l64)
        # the update of this iteration vs the fp64 oracle's (lock step): per tensor at iteration 0;
        # at iteration 1 (chaotic: every fp32 run lands somewhere else) over the whole update
        e_gpu_all = e_cpu_all = 0.0
        for n, p in tr.model.named_parameters():
            if not p.requires_grad:
                continue
            du = p.detach().cpu().double() - p_before[n].double()
            dr = model.params[n].detach().double() - c_before[n].double()
            d64 = m64.params[n].detach() - s_before[n]
            if d64.abs().max() == 0:
                assert du.abs().max() == 0 and dr.abs().max() == 0, n
                continue
            e_gpu, e_cpu = (du - d64).norm().item(), (dr - d64).norm().item()
            e_gpu_all += e_gpu ** 2
            e_cpu_all += e_cpu ** 2
            if it == 0:
                assert e_gpu <= max(3 * e_cpu, 1e-3 * d64.norm().item()), (it, n, e_gpu, e_cpu)
        assert e_gpu_all <= 4 * e_cpu_all, (it, e_gpu_all ** 0.5, e_cpu_all ** 0.5)
    ps = np.array([p.detach().double().sum().item() for p in tr.model.parameters()])
    pc = np.array([model.params[n].double().sum().item() for n in model.names])
    p64 = np.array([m64.params[n].sum().item() for n in m64.names])
    gs = g["src_param_sum"]
    spread = np.maximum(np.abs(pc - p64), np.abs(gs - p64))  # the two fp32 CPU runs around fp64
    assert np.abs(ps - p64).sum() <= 3 * spread.sum() + 1e-6 * np.abs(p64).sum(), \
        (np.abs(ps - p64).sum(), spread.sum())


# ----------------------------------------------------------------------------- 10-iteration loss curve
def test_uda_loss_curve_10_iterations_resynced():
    """Ten fp32 UDA iterations (IW-MaxSquare + multi-level guidance, lambda_t 0.09: configs[3]'s
    losses at 512x256), the oracle re-synced to the GPU state before every iteration so each
    iteration's losses differ by rounding only: loss_seg / loss_target within 1e-3, the guidance CE
    within 1e-3 plus its threshold slack, the IW histogram within 0.1 % of the pixels."""
    from test_gpu_model import _args, _guidance_slack
    tr = _args_trainer(_args)
    cfg = dict(lr=2.5e-4, iter_max=200000, lambda_seg=0.1, IW_ratio=0.2, threshold=0.95,
               target_mode="IW_maxsquare", multi=True, lambda_target=0.09)
    model = orc.Model({k: v.cpu().clone() for k, v in tr.model.state_dict().items()})
    opt = orc.SGDMult(model.params, model.names, cfg["lr"])
    curve = []
    for it in range(10):
        _resync(tr, model, opt)
        xs, ys = synthetic_image(H, W, 20 + it), synthetic_labels(H, W, 19, 20 + it)
        xt = synthetic_image(H, W, 520 + it)
        tr.uda_step(xs.to(DEV), ys.to(DEV), xt.to(DEV))
        torch.cuda.synchronize()
        slack = _guidance_slack(model, xt, cfg["threshold"], cfg["lambda_seg"] * cfg["lambda_target"])
        out = orc.uda_step(model, opt, xs, ys, xt, cfg, it)
        mine = {"loss_seg": tr.loss_val.item(), "loss_target": tr.loss_target.item(),
                "loss_target_2": tr.loss_target_2.item()}
        for k, v in mine.items():
            ab = slack if k == "loss_target_2" else 0.0
            assert v == pytest.approx(out[k], rel=1e-3, abs=ab), f"{k} it{it} (slack {ab:.3g})"
        h = tr.target_loss.last_hist.cpu().numpy().astype(np.int64)
        assert np.abs(h - out["hist"]).sum() <= 2 * 0.001 * H * W, f"hist it{it}"
        curve.append((mine["loss_seg"], mine["loss_target"]))
    assert all(np.isfinite(curve).ravel())


def _args_trainer(_args):
    from maxsquareloss_amd.tools.solve_gta5 import UDATrainer
    tr = UDATrainer(_args(["--target_mode", "IW_maxsquare", "--multi", "True", "--lambda_target", "0.09"]), cuda=True)
    tr.args.iter_max = 200000
    tr.optimizer.zero_grad()
    return tr


# ----------------------------------------------------------------------------- input pipeline
def test_preprocess_kernels_on_reference_kat():
    """csrc/preprocess.hip vs the reference's own _img_transform / id2trainId outputs
    (preprocess_kat.npz): byte-exact, vectorised (w % 4 == 0) and scalar widths, with and
    without the horizontal mirror, every loader table and class subset."""
    from maxsquareloss_amd.utils import preprocess as pp
    g = gold("preprocess_kat.npz")
    for tag in ("a", "b", "c"):
        rgb = torch.from_numpy(g[f"{tag}_rgb"]).to(DEV)
        ids = torch.from_numpy(g[f"{tag}_ids"]).to(DEV)
        for m in (0, 1):
            img = pp.image_transform(rgb, mirror=bool(m), mean=g["img_mean"])
            assert torch.equal(img.cpu()[0], torch.from_numpy(g[f"{tag}_m{m}_img"])), (tag, m)
            for ds in ("cityscapes", "gta5", "synthia"):
                for cls in ("19", "16", "13"):
                    key = f"{tag}_m{m}_{ds}_{cls}"
                    if key not in g.files:
                        continue
                    lab = pp.label_transform(ids, pp.build_lut(ds, cls == "16", cls == "13"), mirror=bool(m))
                    assert lab.dtype == torch.int64
                    assert torch.equal(lab.cpu()[0], torch.from_numpy(g[key]).long()), key
    # the synthetic generator's own images through the device path equal the host path
    from maxsquareloss_amd.utils.synthetic import synthetic_rgb
    rgb = synthetic_rgb(64, 128, 3)
    assert torch.equal(pp.image_transform(torch.from_numpy(rgb).to(DEV)).cpu(), synthetic_image(64, 128, 3))
