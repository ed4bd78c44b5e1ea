"""Image pairs (GPU only): the trunk ops on a (1, C, 2, H, W) batch ([C][2][H][W]) against the same
ops on each image alone.

The trainer runs the source and target images of a UDA iteration as one pair (model.forward_pair,
solve_gta5.py --pair): every conv GEMM once over both images, every BatchNorm with each image's own
bs=1 statistics.  Held here:
  - convs (3x3 dilated, the two-branch ASPP, pointwise, the stem) in every fp32 form and the fp16
    math: outputs and both gradients against fp64 per image, at the same bars as the single-image
    op tests (tests/test_gpu_ops.py), on odd map sizes and dilations whose taps reach across the
    seam between the images (a read from the other image would be a large error);
  - BatchNorm (fused and split kernels): bit-identical to two single-image calls in order -
    outputs, saved statistics, running statistics (source then target), num_batches_tracked,
    input / residual gradients, and dgamma / dbeta (= the second call accumulating into the first);
  - maxpool, subsample: bit-identical per image;
  - the model: forward_pair = forward per image (eval 1e-5; train 1e-3, the bar the single-image
    forward is held to against the oracle: the pair's GEMMs split the doubled pixel axis at other stream-K
    points, i.e. another fp32 summation order, which train-mode bs=1 BatchNorm over 104 layers amplifies -
    3.7e-4 measured), and one UDA iteration with --pair against the two-pass iteration (losses 1e-4, BN
    running statistics 1e-4).
"""
import copy

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from maxsquareloss_amd import ops  # noqa: E402

DEV = "cuda"


@pytest.fixture(params=["mfma_f32", "bf16x6", "f16x3"])
def f32_form(request):
    prev = ops.set_f32_form(request.param)
    yield request.param
    ops.set_f32_form(prev)


def _pair(c, h, w, g, relu=True):
    t = torch.randn(1, c, 2, h, w, generator=g)
    return torch.relu(t) if relu else t


def _img(t, i):
    """Image i of a (1,C,2,H,W) pair as (1,C,H,W) fp64 on the host."""
    return t.detach()[:, :, i].double().cpu().contiguous()


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return (a - b).abs().max().item() / max(b.abs().max().item(), 1e-30)


def _conv_check(fn, ref, x, weights, gy, bar):
    """fn(x, *weights) on the pair vs ref(image, *weights) per image in fp64: y and dx per image,
    dW (and db) against the sum over both images."""
    xg = x.to(DEV).requires_grad_()
    wg = [w.to(DEV).requires_grad_() for w in weights]
    y = fn(xg, *wg)
    y.backward(gy.to(DEV))
    torch.cuda.synchronize()
    wr = [w.double().requires_grad_() for w in weights]
    for i in range(2):
        xr = _img(x, i).requires_grad_()
        yr = ref(xr, *wr)
        yr.backward(_img(gy, i))
        assert _rel(y[:, :, i], yr) < bar, ("y", i)
        assert _rel(xg.grad[:, :, i], xr.grad) < bar, ("dx", i)
    for a, b in zip(wg, wr):
        assert _rel(a.grad, b.grad) < bar, "dW"


@pytest.mark.parametrize("cin,cout,h,w,d", [(256, 256, 17, 33, 2), (64, 64, 33, 65, 1), (512, 512, 9, 17, 4),
                                            (128, 128, 13, 29, 2), (256, 256, 65, 129, 2)])
def test_dconv_pair(cin, cout, h, w, d, f32_form):
    g = torch.Generator().manual_seed(cin + h)
    x, gy = _pair(cin, h, w, g), torch.randn(1, cout, 2, h, w, generator=g)
    wt = torch.randn(cout, cin, 3, 3, generator=g) * 0.05
    cache = ops.PackCache()
    _conv_check(lambda xx, ww: ops.dconv3x3(xx, ww, d, cache),
                lambda xx, ww: F.conv2d(xx, ww, padding=d, dilation=d), x, [wt], gy, 1e-5)


@pytest.mark.parametrize("cin,c,h,w", [(2048, 19, 33, 65), (1024, 16, 17, 33), (96, 13, 9, 17)])
def test_aspp2_pair(cin, c, h, w, f32_form):
    g = torch.Generator().manual_seed(cin + c)
    x, gy = _pair(cin, h, w, g), torch.randn(1, c, 2, h, w, generator=g)
    w0, w1 = torch.randn(c, cin, 3, 3, generator=g) * 0.01, torch.randn(c, cin, 3, 3, generator=g) * 0.01
    b0, b1 = torch.randn(c, generator=g), torch.randn(c, generator=g)
    cache = ops.PackCache()

    def ref(xx, a0, a1, c0, c1):
        return (F.conv2d(xx, a0, c0, padding=6, dilation=6) + F.conv2d(xx, a1, c1, padding=12, dilation=12))

    _conv_check(lambda xx, a0, a1, c0, c1: ops.aspp2(xx, a0, c0, a1, c1, 6, 12, cache), ref, x, [w0, w1, b0, b1],
                gy, 1e-5)


@pytest.mark.parametrize("cin,cout,h,w", [(256, 1024, 17, 33), (1024, 256, 33, 65), (64, 256, 33, 65),
                                          (2048, 512, 9, 17)])
def test_pconv_pair(cin, cout, h, w, f32_form):
    g = torch.Generator().manual_seed(cin * 3 + cout)
    x, gy = _pair(cin, h, w, g), torch.randn(1, cout, 2, h, w, generator=g)
    wt = torch.randn(cout, cin, 1, 1, generator=g) * 0.05
    cache = ops.PackCache(pointwise=True)
    _conv_check(lambda xx, ww: ops.pconv(xx, ww, cache), lambda xx, ww: F.conv2d(xx, ww), x, [wt], gy, 1e-5)


@pytest.mark.parametrize("h,w", [(64, 128), (33, 47)])
def test_stem_conv_pair(h, w, f32_form):
    g = torch.Generator().manual_seed(h * w)
    x = torch.randn(1, 3, 2, h, w, generator=g) * 50
    wt = torch.randn(64, 3, 7, 7, generator=g) * 0.05
    ho, wo = (h + 6 - 7) // 2 + 1, (w + 6 - 7) // 2 + 1
    gy = torch.randn(1, 64, 2, ho, wo, generator=g)
    cache = ops.PackCache(pointwise=True)
    _conv_check(lambda xx, ww: ops.stem_conv(xx, ww, 2, 3, cache), lambda xx, ww: F.conv2d(xx, ww, stride=2, padding=3),
                x, [wt], gy, 1e-5)


@pytest.mark.parametrize("kind,cin,cout,h,w,d", [("3x3", 256, 256, 17, 33, 2), ("aspp", 2048, 16, 17, 33, 6),
                                                 ("1x1", 1024, 256, 17, 33, 0)])
def test_fp16_math_pair(kind, cin, cout, h, w, d):
    """The fp16 conv math (configs[4]) on pairs: per image within the fp16 single-image bar of
    tests/test_gpu_ops.py::test_conv_fp16_math (operands rounded to fp16 once: ~2^-11 relative)."""
    g = torch.Generator().manual_seed(cin + cout + h)
    x, gy = _pair(cin, h, w, g), torch.randn(1, cout, 2, h, w, generator=g)
    ops.set_conv_math("fp16")
    try:
        if kind == "1x1":
            wt = torch.randn(cout, cin, 1, 1, generator=g) * 0.05
            cache = ops.PackCache(pointwise=True)
            _conv_check(lambda xx, ww: ops.pconv(xx, ww, cache), lambda xx, ww: F.conv2d(xx, ww), x, [wt], gy, 4e-3)
        elif kind == "3x3":
            wt = torch.randn(cout, cin, 3, 3, generator=g) * 0.05
            cache = ops.PackCache()
            _conv_check(lambda xx, ww: ops.dconv3x3(xx, ww, d, cache),
                        lambda xx, ww: F.conv2d(xx, ww, padding=d, dilation=d), x, [wt], gy, 4e-3)
        else:
            w0, w1 = torch.randn(cout, cin, 3, 3, generator=g) * 0.01, torch.randn(cout, cin, 3, 3, generator=g) * 0.01
            b0, b1 = torch.randn(cout, generator=g), torch.randn(cout, generator=g)
            cache = ops.PackCache()

            def ref(xx, a0, a1, c0, c1):
                return F.conv2d(xx, a0, c0, padding=6, dilation=6) + F.conv2d(xx, a1, c1, padding=12, dilation=12)

            _conv_check(lambda xx, a0, a1, c0, c1: ops.aspp2(xx, a0, c0, a1, c1, 6, 12, cache), ref, x,
                        [w0, w1, b0, b1], gy, 4e-3)
    finally:
        ops.set_conv_math("fp32")


@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("c,h,w,res,relu", [(256, 65, 129, True, True), (64, 129, 257, False, True),
                                            (1024, 33, 65, False, False), (64, 256, 512, False, True),
                                            (256, 96, 161, False, True), (128, 96, 161, True, True)])
def test_bn_pair_bit_identical(c, h, w, res, relu, fused):
    prev = ops.set_bn_fused(fused)
    try:
        g = torch.Generator().manual_seed(c + h)
        x = (torch.randn(1, c, 2, h, w, generator=g) * 3 + 1).to(DEV)
        r = torch.randn(1, c, 2, h, w, generator=g).to(DEV) if res else None
        gy = torch.randn(1, c, 2, h, w, generator=g).to(DEV)
        bn = nn.BatchNorm2d(c).to(DEV).train()
        with torch.no_grad():
            bn.weight.uniform_(0.5, 1.5)
            bn.bias.normal_()
            bn.running_mean.normal_()
        bn1 = copy.deepcopy(bn)
        xp = x.clone().requires_grad_()
        rp = r.clone().requires_grad_() if res else None
        yp = ops.bn_act(bn, xp, residual=rp, relu=relu)
        yp.backward(gy)
        ys, dxs, drs = [], [], []
        for i in range(2):
            xi = x[:, :, i].contiguous().requires_grad_()
            ri = r[:, :, i].contiguous().requires_grad_() if res else None
            yi = ops.bn_act(bn1, xi, residual=ri, relu=relu)
            yi.backward(gy[:, :, i].contiguous())
            ys.append(yi.detach())
            dxs.append(xi.grad)
            drs.append(ri.grad if res else None)
        torch.cuda.synchronize()
        for i in range(2):
            assert torch.equal(yp.detach()[:, :, i], ys[i]), ("y", i)
            assert torch.equal(xp.grad[:, :, i], dxs[i]), ("dx", i)
            if res:
                assert torch.equal(rp.grad[:, :, i], drs[i]), ("dres", i)
        assert torch.equal(bn.running_mean, bn1.running_mean)
        assert torch.equal(bn.running_var, bn1.running_var)
        assert int(bn.num_batches_tracked) == int(bn1.num_batches_tracked) == 2
        assert torch.equal(bn.weight.grad, bn1.weight.grad)
        assert torch.equal(bn.bias.grad, bn1.bias.grad)
    finally:
        ops.set_bn_fused(prev)


def test_pools_pair_bit_identical():
    g = torch.Generator().manual_seed(5)
    x = torch.randn(1, 64, 2, 129, 257, generator=g).to(DEV)
    x[0, 3, 1, 0, :8] = float("nan")
    for fn in (lambda t: ops.maxpool2d(t, 3, 2, 1, True), lambda t: ops.subsample(t, 2)):
        xp = x.clone().requires_grad_()
        yp = fn(xp)
        gy = torch.randn(yp.shape, generator=g).to(DEV)
        yp.backward(gy)
        for i in range(2):
            xi = x[:, :, i].contiguous().requires_grad_()
            yi = fn(xi)
            yi.backward(gy[:, :, i].contiguous())
            assert torch.equal(yp.detach()[:, :, i].nan_to_num(7.0), yi.detach().nan_to_num(7.0))
            assert torch.equal(xp.grad[:, :, i], xi.grad)


def _trainer(h, w, mode, multi, pair):
    from maxsquareloss_amd.tools.solve_gta5 import UDATrainer, build_parser
    from maxsquareloss_amd.tools.train_source import init_args
    argv = ["--crop_size", f"{w},{h}", "--target_crop_size", f"{w},{h}", "--imagenet_pretrained", "False",
            "--save_dir", "", "--num_classes", "19", "--target_mode", mode, "--multi", str(multi),
            "--lambda_target", "0.1", "--iter_max", "200000", "--pair", str(pair)]
    args, _, _ = init_args(build_parser().parse_args(argv))
    return UDATrainer(args, cuda=True)


@pytest.mark.parametrize("train", [True, False])
def test_forward_pair_matches_forward(train):
    """Train mode: per-image batch statistics, running statistics updated source then target
    (forward_pair on one copy of the model, two forwards on another); eval: running statistics."""
    tr = _trainer(256, 512, "maxsquare", False, True)
    from maxsquareloss_amd.utils.synthetic import synthetic_image
    xs, xt = synthetic_image(256, 512, 3).to(DEV), synthetic_image(256, 512, 503).to(DEV)
    m = tr.model.train(train)
    m1 = copy.deepcopy(m)
    with torch.no_grad():
        outs = m.forward_pair(xs, xt)
        single = [m1(xs), m1(xt)]
    torch.cuda.synchronize()
    bar = 1e-3 if train else 1e-5
    for (p2, p1), (s2, s1) in zip(outs, single):
        assert _rel(p2, s2) < bar and _rel(p1, s1) < bar
    for (n, a), b in zip(m.named_buffers(), m1.buffers()):
        if "running" in n:
            assert _rel(a, b) < bar, n


@pytest.mark.parametrize("mode,multi", [("maxsquare", False), ("IW_maxsquare", True)])
def test_pair_step_matches_two_pass_step(mode, multi):
    from maxsquareloss_amd.utils.synthetic import synthetic_image, synthetic_labels
    h, w = 256, 512
    xs, ys = synthetic_image(h, w, 11).to(DEV), synthetic_labels(h, w, 19, 11).to(DEV)
    xt = synthetic_image(h, w, 511).to(DEV)
    res = []
    for pair in (True, False):
        tr = _trainer(h, w, mode, multi, pair)
        tr.optimizer.zero_grad()
        tr.uda_step(xs, ys, xt)
        torch.cuda.synchronize()
        vals = [tr.loss_val.item(), tr.loss_target.item()] + ([tr.loss_target_2.item()] if multi else [])
        bufs = {n: b.detach().clone() for n, b in tr.model.named_buffers() if "running" in n}
        res.append((vals, bufs))
    # the guidance CE (multi) thresholds and argmaxes per pixel: 1e-3 for the few decisions that sit
    # within rounding of their threshold (tests/test_gpu_configs.py holds it to the oracle)
    for k, (a, b) in enumerate(zip(res[0][0], res[1][0])):
        assert a == pytest.approx(b, rel=1e-4 if k < 2 else 1e-3, abs=1e-6), k
    for n in res[0][1]:
        assert _rel(res[0][1][n], res[1][1][n]) < 1e-4, n
