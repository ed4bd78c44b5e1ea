"""Conv -> BN fusion (GPU only; SURVEY.md §8f row 1, deeplab_multi.py:12-46).

With ops.FOLD the forward-form conv GEMMs leave the stream-K pieces of their split tiles for the BN
kernel that consumes the map (msl_*_pend + msl_bn_fwd_pend / msl_bn_bwd_pend).  The BN kernels sum
the pieces in k_sk_reduce's own order, so everything is held BIT-IDENTICAL to the unfused path
(ops.FOLD = False):
  - single conv -> BN chains through the ops, every conv kind the trunk has (pointwise with and without
    data-parallel rounds, accumulate epilogue, 3x3 register-B and pre-split forms, a 64-row GEMM whose BN
    runs the split kernels so the output is finished by msl_sk_finish instead), f16x3 and fp16;
  - a whole UDA training iteration (forward, backward, SGD) at two sizes, f16x3 and fp16: losses, every
    parameter, every BN buffer - and the folds were taken;
  - a pending output read by an op that does not fold is finished first; a pending gradient that
    autograd modified (an edge wrongly marked foldable) raises instead of computing garbage.
"""
import copy

import pytest
import torch
import torch.nn as nn

pytestmark = pytest.mark.gpu

from maxsquareloss_amd import hip, ops  # noqa: E402

DEV = "cuda"


@pytest.fixture(params=["fp32", "fp16"])
def math(request):
    prev = ops.CONV_MATH
    ops.set_conv_math(request.param)
    yield request.param
    ops.set_conv_math(prev)


class _Count:
    """Counts the folds taken (ops._take_pend hits)."""

    def __init__(self, monkeypatch):
        self.pend = 0
        take = ops._take_pend

        def take_c(t):
            r = take(t)
            self.pend += r is not None
            return r

        monkeypatch.setattr(ops, "_take_pend", take_c)


def _chain(kind, cin, cout, h, w, d, fold, seed, res):
    """x -> conv(fold) -> bn_act (+residual, ReLU) -> weighted sum; returns y and every gradient."""
    g = torch.Generator().manual_seed(seed)
    x = torch.relu(torch.randn(1, cin, 2, h, w, generator=g)).to(DEV).requires_grad_()
    k = 3 if kind == "3x3" else 1
    wt = (torch.randn(cout, cin, k, k, generator=g) * (0.5 / (cin * k * k) ** 0.5)).to(DEV).requires_grad_()
    r = torch.randn(1, cout, 2, h, w, generator=g).to(DEV) if res else None
    gy = torch.randn(1, cout, 2, h, w, generator=g).to(DEV)
    bn = nn.BatchNorm2d(cout).to(DEV).train()
    with torch.no_grad():
        bn.weight.copy_(torch.rand(cout, generator=g) + 0.5)
        bn.bias.copy_(torch.randn(cout, generator=g))
    cache = ops.PackCache(pointwise=kind != "3x3")
    # the conv reads a BN output that nothing else reads, so its data gradient may reach that BN's
    # backward unfinished (fold bit 1), as conv2 / conv3 in a Bottleneck
    bn0 = nn.BatchNorm2d(cin).to(DEV).train()
    xin = ops.bn_act(bn0, x, relu=True)
    if kind == "3x3":
        y = ops.dconv3x3(xin, wt, d, cache, fold)
    else:
        y = ops.pconv(xin, wt, cache, None, fold)
    out = ops.bn_act(bn, y, residual=r, relu=True)
    out.backward(gy)
    torch.cuda.synchronize()
    return [out.detach(), y.detach(), x.grad, wt.grad, bn.weight.grad, bn.bias.grad, bn0.weight.grad,
            bn.running_mean, bn.running_var]


@pytest.mark.parametrize("kind,cin,cout,h,w,d,res,folds", [
    ("1x1", 256, 1024, 65, 129, 0, True, 2),    # 1056 tiles: data-parallel rounds + stream-K remainder
    ("1x1", 1024, 256, 65, 129, 0, False, 2),   # pure stream-K
    ("1x1", 512, 2048, 33, 65, 0, True, 1),    # its data gradient leaves > 4 pieces per tile
    ("3x3", 256, 256, 65, 129, 2, False, 2),    # the bench's dominant op (image operand in registers)
    ("3x3", 512, 512, 33, 65, 4, False, 0),     # the pre-split (BP) form; > 4 pieces per tile: reduced by the GEMM call
    ("3x3", 128, 128, 65, 129, 1, False, 0),    # 5 pieces per tile
    ("1x1", 256, 64, 129, 257, 0, False, 1),    # 64-row tiles; a 64-channel 33k-px BN: split kernels, finished first
])
def test_conv_bn_chain_bit_identical(kind, cin, cout, h, w, d, res, folds, math, monkeypatch):
    ref = _chain(kind, cin, cout, h, w, d, 0, cin + cout + h, res)
    cnt = _Count(monkeypatch)
    got = _chain(kind, cin, cout, h, w, d, 3, cin + cout + h, res)
    for i, (a, b) in enumerate(zip(got, ref)):
        assert torch.equal(a, b), i
    # the forward and the data gradient each leave a pending map where the schedule allows it
    assert cnt.pend >= folds, cnt.pend


def _trainer(h, w, math_, fold):
    from maxsquareloss_amd.tools.solve_gta5 import UDATrainer, build_parser
    from maxsquareloss_amd.tools.train_source import init_args
    argv = ["--crop_size", f"{w},{h}", "--target_crop_size", f"{w},{h}", "--imagenet_pretrained", "False",
            "--save_dir", "", "--num_classes", "19", "--target_mode", "IW_maxsquare", "--multi", "True",
            "--lambda_target", "0.1", "--iter_max", "200000", "--conv_math", math_]
    args, _, _ = init_args(build_parser().parse_args(argv))
    ops.FOLD = fold
    try:
        return UDATrainer(args, cuda=True)
    finally:
        ops.FOLD = True


@pytest.mark.parametrize("h,w", [(256, 512), (512, 1024)])
def test_uda_step_fold_bit_identical(h, w, math, monkeypatch):
    from maxsquareloss_amd.utils.synthetic import synthetic_image, synthetic_labels
    xs, ys = synthetic_image(h, w, 21).to(DEV), synthetic_labels(h, w, 19, 21).to(DEV)
    xt = synthetic_image(h, w, 521).to(DEV)
    res = []
    for fold in (False, True):
        torch.manual_seed(0)
        tr = _trainer(h, w, math, fold)
        if res:  # the same initial weights
            tr.model.load_state_dict(res[0][2])
        init = copy.deepcopy(tr.model.state_dict())
        cnt = _Count(monkeypatch) if fold else None
        ops.FOLD = fold
        try:
            tr.uda_step(xs, ys, xt)
            torch.cuda.synchronize()
        finally:
            ops.FOLD = True
            monkeypatch.undo()
        vals = [tr.loss_val.item(), tr.loss_target.item(), tr.loss_target_2.item()]
        res.append((vals, {k: v.detach().clone() for k, v in tr.model.state_dict().items()}, init, cnt))
    (v0, s0, _, _), (v1, s1, _, cnt) = res
    assert v0 == v1, (v0, v1)
    for k in s0:
        assert torch.equal(s0[k], s1[k]), k
    # every Bottleneck conv output with a fused-form BN (layers 1-4: 99 convs, minus layer1's 64-channel
    # maps) and most data gradients fold
    assert cnt.pend > 100, cnt.pend


def test_pending_output_finished_for_other_consumers():
    """A folded conv output read by an op that does not fold (here maxpool) is completed first."""
    g = torch.Generator().manual_seed(3)
    x = torch.randn(1, 1024, 2, 65, 129, generator=g).to(DEV)
    wt = (torch.randn(256, 1024, 1, 1, generator=g) * 0.03).to(DEV)
    outs = []
    for fold in (0, 1):
        y = ops.pconv(x, wt, ops.PackCache(pointwise=True), None, fold)
        if fold:
            assert getattr(y, "_msl_pend", None) is not None
        outs.append(ops.maxpool2d(y, 3, 2, 1, True))
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])


def test_modified_pending_gradient_raises():
    """An edge wrongly marked foldable: autograd sums a second gradient into the pending dx in place
    (its version counter moves) - the BN backward refuses it rather than reading a corrupt map.  (Only
    this order is detectable: the later-created conv's backward runs first and its dx is the buffer
    autograd accumulates into.  The model's flags are what keeps such edges out.)"""
    g = torch.Generator().manual_seed(4)
    x = torch.randn(1, 256, 2, 33, 65, generator=g).to(DEV).requires_grad_()
    bn0 = nn.BatchNorm2d(256).to(DEV).train()
    wt = (torch.randn(1024, 256, 1, 1, generator=g) * 0.05).to(DEV).requires_grad_()
    cache = ops.PackCache(pointwise=True)
    xin = ops.bn_act(bn0, x, relu=True)
    y = ops.pconv(xin, wt, cache, None, 0) + ops.pconv(xin, wt, cache, None, 3)  # xin has two consumers
    with pytest.raises(hip.MSLError):
        y.sum().backward()
