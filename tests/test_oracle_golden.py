"""CPU: pin the oracle (oracle/msl_oracle.py) against the reference's own outputs.

tests/golden/*.npz were produced by oracle/gen_golden.py from the reference's
deeplab_multi.py / loss.py imported by path (survey container only).  The
oracle then serves as the checker of the HIP path on the GPU box, where the
reference does not exist.
"""
import json
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import msl_oracle as orc
from maxsquareloss_amd.utils.synthetic import counter_normal, init_weights, synthetic_image, synthetic_labels

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def gold(name):
    return np.load(os.path.join(GOLD, name), allow_pickle=False)


@pytest.mark.parametrize("C", [19, 16, 13])
def test_loss_kat(C):
    g = gold("loss_kat.npz")
    low = torch.from_numpy(g[f"C{C}_low"])
    low2 = torch.from_numpy(g[f"C{C}_low2"])
    y = torch.from_numpy(g[f"C{C}_y"])
    hw = (64, 128)
    up = lambda t: F.interpolate(t, size=hw, mode="bilinear", align_corners=True)  # noqa: E731
    # MaxSquare
    lr = low.clone().requires_grad_()
    l = orc.maxsquare(F.softmax(up(lr), 1))
    l.backward()
    assert l.item() == pytest.approx(float(g[f"C{C}_ms"]), rel=1e-6)
    np.testing.assert_allclose(lr.grad.numpy(), g[f"C{C}_ms_dlow"], rtol=1e-5, atol=1e-9)
    # IW MaxSquare: histogram bit-exact
    lr = low.clone().requires_grad_()
    l, hist = orc.iw_maxsquare(F.softmax(up(lr), 1), 0.2, C)
    l.backward()
    assert np.array_equal(hist.numpy().astype(np.int64), g[f"C{C}_iw_hist"])
    assert l.item() == pytest.approx(float(g[f"C{C}_iw"]), rel=1e-6)
    np.testing.assert_allclose(lr.grad.numpy(), g[f"C{C}_iw_dlow"], rtol=1e-5, atol=1e-9)
    # CE
    lr = low.clone().requires_grad_()
    l = orc.ce(up(lr), y)
    l.backward()
    assert l.item() == pytest.approx(float(g[f"C{C}_ce"]), rel=1e-6)
    np.testing.assert_allclose(lr.grad.numpy(), g[f"C{C}_ce_dlow"], rtol=1e-5, atol=1e-9)
    # multi-level guidance
    for thr in (0.95, 0.5):
        t = str(thr).replace(".", "p")
        lr = low.clone().requires_grad_()
        lab = orc.multi_guidance_label(F.softmax(up(low2), 1), F.softmax(up(lr), 1), thr)
        assert np.array_equal(lab.numpy().astype(np.int8), g[f"C{C}_multi{t}_label"])
        l = orc.multi_guidance_ce(up(low2), up(lr), thr)
        want = float(g[f"C{C}_multi{t}_ce"])
        if np.isnan(want):
            assert np.isnan(l.item())
            continue
        l.backward()
        assert l.item() == pytest.approx(want, rel=1e-6)
        np.testing.assert_allclose(lr.grad.numpy(), g[f"C{C}_multi{t}_dlow"], rtol=1e-5, atol=1e-9)


def test_loss_edge_cases():
    g = gold("loss_kat.npz")
    tie = torch.from_numpy(g["tie_logits"])
    P = F.softmax(tie, 1)
    _, arg = torch.max(P, 1)
    assert np.array_equal(arg.numpy().astype(np.int8), g["tie_argmax"])  # first max wins
    l, _ = orc.iw_maxsquare(P, 0.2, 19)
    assert l.item() == pytest.approx(float(g["tie_iw"]), rel=1e-6)
    l = orc.ce(torch.zeros(1, 19, 4, 8), torch.full((1, 4, 8), -1))
    assert np.isnan(l.item()) and np.isnan(float(g["allignored_ce"]))  # quirk Q8


def _chk(t, g, prefix, rtol=1e-5):
    a = t.detach().double().numpy()
    flat = a.reshape(-1)
    np.testing.assert_allclose(flat[g[prefix + "_idx"]], g[prefix + "_sample"], rtol=rtol, atol=rtol * np.abs(flat).max())
    assert a.sum() == pytest.approx(float(g[prefix + "_sum"]), rel=rtol, abs=rtol * float(g[prefix + "_abssum"]))


def test_conv_kat():
    g = gold("conv_kat.npz")
    h, w = 17, 33
    for name, planes, dil in (("d2", 256, 2), ("d4", 512, 4)):
        wt = torch.from_numpy(counter_normal(5, f"conv_{name}_w", planes * planes * 9, 0.01)).view(planes, planes, 3, 3).requires_grad_()
        x = torch.from_numpy(counter_normal(6, f"conv_{name}_x", planes * h * w)).view(1, planes, h, w).requires_grad_()
        gy = torch.from_numpy(counter_normal(7, f"conv_{name}_gy", planes * h * w)).view(1, planes, h, w)
        y = F.conv2d(x, wt, padding=dil, dilation=dil)
        y.backward(gy)
        _chk(y, g, f"{name}_y")
        _chk(x.grad, g, f"{name}_dx")
        _chk(wt.grad, g, f"{name}_dw")
    for head, cin in (("aspp5", 1024), ("aspp6", 2048)):
        params = {}
        for i in range(4):
            params[f"{head}.conv2d_list.{i}.weight"] = torch.from_numpy(
                counter_normal(8, f"{head}_w{i}", 19 * cin * 9, 0.01)).view(19, cin, 3, 3).requires_grad_()
            params[f"{head}.conv2d_list.{i}.bias"] = torch.from_numpy(counter_normal(9, f"{head}_b{i}", 19, 0.01)).requires_grad_()
        x = torch.from_numpy(counter_normal(10, f"{head}_x", cin * h * w)).view(1, cin, h, w).requires_grad_()
        gy = torch.from_numpy(counter_normal(11, f"{head}_gy", 19 * h * w)).view(1, 19, h, w)
        y = orc._aspp(x, params, head)
        y.backward(gy)
        _chk(y, g, f"{head}_y")
        _chk(x.grad, g, f"{head}_dx")
        for i in range(4):
            wgt = params[f"{head}.conv2d_list.{i}.weight"]
            assert (wgt.grad is not None) == bool(g[f"{head}_w{i}_hasgrad"])  # Q1: only branches 0, 1
            if wgt.grad is not None:
                _chk(wgt.grad, g, f"{head}_dw{i}")
                np.testing.assert_allclose(params[f"{head}.conv2d_list.{i}.bias"].grad.numpy(), g[f"{head}_db{i}"], rtol=1e-5)


def test_sgd_kat_oracle_semantics():
    """The oracle's SGD restatement == torch.optim.SGD(foreach=False) on duplicated lists."""
    g = gold("sgd_kat.npz")
    mult = list(g["mult"])
    params = [torch.from_numpy(g[f"p{i}_init"]).clone() for i in range(len(mult))]
    bufs = [None] * len(params)
    for step in range(3):
        grads = [torch.from_numpy(g[f"g{i}_step{step}"]) if i < 4 else None for i in range(len(params))]
        # restated single-tensor loop (msl_oracle.SGDMult.step, per parameter)
        for i, (p, k) in enumerate(zip(params, mult)):
            if grads[i] is None:
                continue
            occ = [bufs[i]] * k
            for r in range(k):
                d = grads[i].add(p, alpha=5e-4)
                if occ[r] is None:
                    occ[r] = d.clone()
                else:
                    occ[r].mul_(0.9).add_(d)
                p.add_(occ[r], alpha=-0.01)
                if bufs[i] is not None:
                    occ = [bufs[i]] * k
            bufs[i] = occ[-1]
        for i, p in enumerate(params):
            np.testing.assert_array_equal(p.numpy(), g[f"p{i}_step{step}"])


def test_optim_lists_match_reference():
    with open(os.path.join(GOLD, "optim_lists.json")) as f:
        ref = json.load(f)
    names = [n for n, _, _ in orc.param_specs(19)]
    g0, g1 = orc.optim_param_lists(names)
    assert g0 == ref["group0"]
    assert g1 == ref["group1"]
    from collections import Counter
    cnt = Counter(g0)
    assert cnt["conv1.weight"] == 1
    assert sum(1 for v in cnt.values() if v == 3) == 297 and sum(1 for v in cnt.values() if v == 4) == 12
    assert len(g0) == 940


def _oracle_model(num_classes=19):
    from maxsquareloss_amd.graphs.models.deeplab_multi import DeeplabMulti
    m = init_weights(DeeplabMulti(num_classes, pretrained=False), 12345)
    return orc.Model(m.state_dict(), num_classes)


@pytest.mark.slow
def test_step_goldens_cfg1():
    """Oracle UDA / source iterations at 512x256 reproduce the reference's loss curve and updates."""
    g = gold("step_cfg1.npz")
    h, w = (int(v) for v in g["hw"])
    torch.set_num_threads(min(8, os.cpu_count()))
    common = dict(lr=2.5e-4, iter_max=200000, lambda_seg=0.1, IW_ratio=0.2, threshold=0.95)
    for tag, cfg in (("ms", dict(target_mode="maxsquare", multi=False, lambda_target=0.1)),
                     ("iwmulti", dict(target_mode="IW_maxsquare", multi=True, lambda_target=0.09))):
        cfg = {**common, **cfg}
        model = _oracle_model()
        opt = orc.SGDMult(model.params, model.names, cfg["lr"])
        for it in range(2):
            xs, ys = synthetic_image(h, w, it), synthetic_labels(h, w, 19, it)
            xt = synthetic_image(h, w, 500 + it)
            out = orc.uda_step(model, opt, xs, ys, xt, cfg, it)
            for k in ("loss_seg", "loss_target", "loss_seg_2", "loss_target_2"):
                key = f"{tag}_it{it}_{k}"
                if key in g.files:
                    assert out[k] == pytest.approx(float(g[key]), rel=1e-4), key
            if f"{tag}_it{it}_hist" in g.files:
                assert np.array_equal(out["hist"], g[f"{tag}_it{it}_hist"])
        ps = np.array([model.params[n].double().sum().item() for n in model.names])
        np.testing.assert_allclose(ps, g[f"{tag}_param_sum"], rtol=1e-4, atol=1e-6)
    model = _oracle_model()
    opt = orc.SGDMult(model.params, model.names, 2.5e-4)
    cfg = dict(common, multi=True)
    for it in range(2):
        x, y = synthetic_image(h, w, 100 + it), synthetic_labels(h, w, 19, 100 + it)
        out = orc.source_step(model, opt, x, y, cfg, it)
        assert out["loss"] == pytest.approx(float(g[f"src_it{it}_loss"]), rel=1e-4)


def test_preprocess_kat():
    """The oracle's loader transforms and the product's id->trainId tables (utils/preprocess.py,
    host side) reproduce the reference's own _img_transform / id2trainId outputs
    (preprocess_kat.npz, written by oracle/gen_golden_preprocess.py)."""
    from maxsquareloss_amd.utils import preprocess as pp
    g = gold("preprocess_kat.npz")
    tables = {"cityscapes": pp.CITYSCAPES_ID_TO_TRAINID, "gta5": pp.GTA5_ID_TO_TRAINID,
              "synthia": pp.SYNTHIA_ID_TO_TRAINID}
    n = 0
    for tag in ("a", "b", "c"):
        rgb, ids = g[f"{tag}_rgb"], g[f"{tag}_ids"]
        for m in (0, 1):
            assert np.array_equal(orc.image_transform(rgb, g["img_mean"], bool(m)), g[f"{tag}_m{m}_img"])
            for ds, table in tables.items():
                for cls in ("19", "16", "13"):
                    key = f"{tag}_m{m}_{ds}_{cls}"
                    if key not in g.files:
                        continue
                    s16 = pp.SET_16 if cls == "16" else None
                    s13 = pp.SET_13 if cls == "13" else None
                    want = g[key]
                    assert np.array_equal(orc.label_transform(ids, table, s16, s13, bool(m)), want), key
                    lut = pp.build_lut(ds, cls == "16", cls == "13")
                    d = ids[:, ::-1] if m else ids
                    assert np.array_equal(lut[d].astype(np.float32), want), key
                    n += 1
    assert n == 3 * 2 * 8


def test_round_f16_is_fp16_rounding_under_a_pow2_scale():
    """oracle.round_f16 (the fp16 path's operand rounding, emulated): the absolute maximum lands in
    [2^14, 2^15) after scaling, every value is an fp16 number times the inverse scale, rounding is to
    nearest (|error| <= half an fp16 ulp of the scaled value), per-row scales along `dim`."""
    g = torch.Generator().manual_seed(3)
    x = torch.randn(4, 7, 5, 6, generator=g) * torch.logspace(-8, 3, 4).view(4, 1, 1, 1)
    for dim in (None, 0, 1):
        r = orc.round_f16(x, dim)
        if dim is None:
            m = x.abs().max().view(1, 1, 1, 1)
        else:
            m = x.abs().transpose(0, dim).reshape(x.shape[dim], -1).max(1)[0]
            m = m.view([-1 if i == dim else 1 for i in range(4)])
        sc = torch.ldexp(torch.ones_like(m), 15 - torch.frexp(m).exponent)
        assert bool(((m * sc >= 2 ** 14) & (m * sc < 2 ** 15)).all())
        s = (r * sc).double()
        assert torch.equal(s, s.half().double())  # representable in fp16
        ulp = torch.ldexp(torch.ones_like(s), torch.frexp((x * sc).abs().clamp_min(2 ** -14)).exponent - 11)
        assert bool(((s - (x * sc).double()).abs() <= ulp.double() / 2 + 1e-30).all())
    assert torch.equal(orc.round_f16(orc.round_f16(x)), orc.round_f16(x))  # idempotent


def test_conv_f16_emulation_rounds_every_product_operand():
    """oracle.conv_f16: forward = conv of the rounded operands; data gradient = transposed conv of the
    rounded dy and W; weight gradient from per-channel-rounded x and dy when the predicate says the
    kernel rounds them, exact otherwise; the bias gradient exact."""
    g = torch.Generator().manual_seed(5)
    x = torch.randn(1, 8, 9, 11, generator=g)
    w = torch.randn(6, 8, 3, 3, generator=g) * 0.01
    b = torch.randn(6, generator=g)
    gy = torch.randn(1, 6, 9, 11, generator=g) * 1e-5
    for rounds in (True, False):
        seen = []
        conv = orc.conv_f16(lambda *a: seen.append(a) or rounds)
        xv, wv, bv = x.clone().requires_grad_(), w.clone().requires_grad_(), b.clone().requires_grad_()
        y = conv(xv, wv, bv, 1, 2, 2)
        assert torch.equal(y, F.conv2d(orc.round_f16(x), orc.round_f16(w), b, 1, 2, 2))
        y.backward(gy)
        assert seen == [(8, 6, 3, 9, 11)]
        gx = torch.nn.grad.conv2d_input(x.shape, orc.round_f16(w), orc.round_f16(gy), 1, 2, 2)
        xr, gr = (orc.round_f16(x, 1), orc.round_f16(gy, 1)) if rounds else (x, gy)
        gw = torch.nn.grad.conv2d_weight(xr, w.shape, gr, 1, 2, 2)
        assert torch.equal(xv.grad, gx) and torch.equal(wv.grad, gw)
        assert torch.equal(bv.grad, gy.sum((0, 2, 3)))
