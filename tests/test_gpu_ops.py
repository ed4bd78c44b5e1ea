"""Kernel-level parity of the HIP path against fp64 / torch-CPU references (GPU only).

Tolerances: conv outputs and gradients within 1e-5 of max|ref|
against an fp64 CPU conv (the kernels are exact fp32 FMA chains, only the
summation order differs); upsample forward bit-exact vs torch-CPU; losses
1e-5 relative; class histograms bit-exact.
"""
import ctypes
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from maxsquareloss_amd import ops  # noqa: E402

DEV = "cuda"


@pytest.fixture(params=["mfma_f32", "bf16x6", "f16x3"])
def f32_form(request):
    """Every matrix-core form of the fp32 convs is held to the same fp64 tolerance."""
    prev = ops.set_f32_form(request.param)
    yield request.param
    ops.set_f32_form(prev)


def _rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return (a - b).abs().max().item() / max(b.abs().max().item(), 1e-30)


def _conv_ref(x, w, d, bias=None):
    return F.conv2d(x.double(), w.double(), None if bias is None else bias.double(), padding=d, dilation=d)


def test_launch_guard_refuses_oversized_blocks():
    """MSL_LAUNCH (r06): a block over the kernel's __launch_bounds__ returns MSL_ERR_LAUNCH (-4) and launches
    nothing; within the bound the kernel runs (the probe kernel is bound to 256 threads)."""
    from maxsquareloss_amd import hip
    lib = hip.load()
    out = torch.full((1024,), -1.0, device=DEV)
    assert lib.msl_launch_guard_probe(512, out.data_ptr(), hip.stream_ptr()) == -4
    assert lib.msl_launch_guard_probe(257, out.data_ptr(), hip.stream_ptr()) == -4
    torch.cuda.synchronize()
    assert (out == -1).all()
    assert lib.msl_launch_guard_probe(256, out.data_ptr(), hip.stream_ptr()) == 0
    torch.cuda.synchronize()
    assert torch.equal(out[:256].cpu(), torch.arange(256, dtype=torch.float32))
    assert (out[256:] == -1).all()


@pytest.mark.parametrize("cin,cout,h,w,d", [
    (256, 256, 17, 33, 2), (512, 512, 17, 33, 4), (64, 64, 33, 65, 1), (32, 48, 9, 13, 2),
    (256, 256, 65, 129, 2)])
def test_dconv_fwd_bwd(cin, cout, h, w, d, f32_form):
    g = torch.Generator().manual_seed(cin * 7 + h)
    x = torch.randn(1, cin, h, w, generator=g)
    wt = torch.randn(cout, cin, 3, 3, generator=g) * 0.05
    gy = torch.randn(1, cout, h, w, generator=g)
    xr, wr = x.double().requires_grad_(), wt.double().requires_grad_()
    yr = F.conv2d(xr, wr, padding=d, dilation=d)
    yr.backward(gy.double())
    xg = x.to(DEV).requires_grad_()
    wg = wt.to(DEV).requires_grad_()
    cache = ops.PackCache()
    y = ops.dconv3x3(xg, wg, d, cache)
    y.backward(gy.to(DEV))
    torch.cuda.synchronize()
    assert _rel(y, yr) < 1e-5
    assert _rel(xg.grad, xr.grad) < 1e-5
    assert _rel(wg.grad, wr.grad) < 1e-5


@pytest.mark.parametrize("cin,cout,h,w", [
    (64, 256, 33, 65), (256, 64, 33, 65), (1024, 256, 17, 33), (48, 160, 9, 13), (512, 2048, 17, 33),
    (2048, 512, 65, 129), (256, 1024, 65, 129)])
def test_pconv_fwd_bwd(cin, cout, h, w, f32_form):
    g = torch.Generator().manual_seed(cin * 3 + cout)
    x = torch.randn(1, cin, h, w, generator=g)
    wt = torch.randn(cout, cin, 1, 1, generator=g) * 0.05
    gy = torch.randn(1, cout, h, w, generator=g)
    xr, wr = x.double().requires_grad_(), wt.double().requires_grad_()
    yr = F.conv2d(xr, wr)
    yr.backward(gy.double())
    xg = x.to(DEV).requires_grad_()
    wg = wt.to(DEV).requires_grad_()
    cache = ops.PackCache(pointwise=True)
    y = ops.pconv(xg, wg, cache)
    y.backward(gy.to(DEV))
    torch.cuda.synchronize()
    assert _rel(y, yr) < 1e-5
    assert _rel(xg.grad, xr.grad) < 1e-5
    assert _rel(wg.grad, wr.grad) < 1e-5
    # an in-place weight update must invalidate the packed copy
    with torch.no_grad():
        wg.mul_(-2.0)
    y2 = ops.pconv(xg.detach(), wg.detach(), cache)
    torch.cuda.synchronize()
    assert _rel(y2, -2.0 * yr.detach()) < 1e-5


@pytest.mark.parametrize("cin,cout,h,w", [(64, 256, 129, 257), (256, 64, 129, 257), (64, 64, 129, 257),
                                           (1024, 256, 65, 129), (256, 1024, 65, 129), (1024, 512, 65, 129),
                                           (512, 128, 65, 129), (128, 512, 65, 129), (512, 2048, 17, 33)])
def test_conv1x1_step_shapes(cin, cout, h, w, f32_form):
    """ops.conv1x1 on every 1x1 shape of the UDA step: all three GEMMs on the HIP pointwise kernels,
    every gradient against fp64, in every fp32 form."""
    g = torch.Generator().manual_seed(cin + 5 * cout)
    x = torch.randn(1, cin, h, w, generator=g)
    wt = torch.randn(cout, cin, 1, 1, generator=g) * 0.05
    gy = torch.randn(1, cout, h, w, generator=g)
    xr, wr = x.double().requires_grad_(), wt.double().requires_grad_()
    yr = F.conv2d(xr, wr)
    yr.backward(gy.double())
    xg = x.to(DEV).requires_grad_()
    wg = wt.to(DEV).requires_grad_()
    y = ops.conv1x1(xg, wg, ops.PackCache(pointwise=True))
    y.backward(gy.to(DEV))
    torch.cuda.synchronize()
    assert _rel(y, yr) < 1e-5
    assert _rel(xg.grad, xr.grad) < 1e-5
    assert _rel(wg.grad, wr.grad) < 1e-5


@pytest.mark.parametrize("cin,c,h,w", [(1024, 19, 17, 33), (2048, 19, 33, 65), (96, 16, 9, 17), (64, 13, 65, 129)])
def test_aspp2_fwd_bwd(cin, c, h, w, f32_form):
    g = torch.Generator().manual_seed(cin + c)
    x = torch.randn(1, cin, h, w, generator=g)
    w0 = torch.randn(c, cin, 3, 3, generator=g) * 0.01
    w1 = torch.randn(c, cin, 3, 3, generator=g) * 0.01
    b0 = torch.randn(c, generator=g) * 0.01
    b1 = torch.randn(c, generator=g) * 0.01
    gy = torch.randn(1, c, h, w, generator=g)
    ref = [t.double().requires_grad_() for t in (x, w0, b0, w1, b1)]
    yr = F.conv2d(ref[0], ref[1], ref[2], padding=6, dilation=6) + F.conv2d(ref[0], ref[3], ref[4], padding=12, dilation=12)
    yr.backward(gy.double())
    dev = [t.to(DEV).requires_grad_() for t in (x, w0, b0, w1, b1)]
    y = ops.aspp2(dev[0], dev[1], dev[2], dev[3], dev[4], 6, 12, ops.PackCache())
    y.backward(gy.to(DEV))
    torch.cuda.synchronize()
    assert _rel(y, yr) < 1e-5
    for a, b in zip(dev, ref):
        assert _rel(a.grad, b.grad) < 1e-5


@pytest.mark.parametrize("cin,c,h,w,n,d0,d1", [(2048, 19, 65, 129, 2, 6, 12), (1024, 16, 96, 161, 2, 6, 12),
                                              (256, 19, 9, 17, 1, 6, 12), (128, 5, 13, 7, 2, 2, 5)])
def test_aspp_shift_form_matches_direct(cin, c, h, w, n, d0, d1, monkeypatch):
    """The r04 shift form of the heads (one pointwise GEMM with 18*C rows, then shifts: csrc/aspp.hip)
    against the two-branch implicit GEMM (ASPP_FORM = "direct") on pairs and single images, incl. maps
    narrower / shorter than the dilation (every tap of some pixels falls outside its image)."""
    g = torch.Generator().manual_seed(cin + c + h)
    shape = (1, cin, n, h, w) if n > 1 else (1, cin, h, w)
    x = torch.randn(shape, generator=g).to(DEV)
    ws = [(torch.randn(c, cin, 3, 3, generator=g) * 0.01).to(DEV) for _ in range(2)]
    bs = [torch.randn(c, generator=g).to(DEV) for _ in range(2)]
    gy = torch.randn((1, c) + shape[2:], generator=g).to(DEV)
    res = []
    for form in ("direct", "shift"):
        monkeypatch.setattr(ops, "ASPP_FORM", form)
        leaves = [t.clone().requires_grad_() for t in (x, ws[0], bs[0], ws[1], bs[1])]
        y = ops.aspp2(*leaves, d0, d1, ops.PackCache())
        y.backward(gy)
        torch.cuda.synchronize()
        res.append([y.detach()] + [t.grad for t in leaves])
    for i, (a, b) in enumerate(zip(*res)):
        assert _rel(a, b) < 1e-5, i


@pytest.mark.parametrize("math", ["bf16", "fp16"])
@pytest.mark.parametrize("cin,c,h,w,n,d0,d1", [(2048, 19, 65, 129, 2, 6, 12), (1024, 16, 96, 161, 2, 6, 12),
                                              (256, 19, 9, 17, 1, 6, 12), (128, 5, 13, 7, 2, 2, 5)])
def test_aspp_shift_form_low_precision(math, cin, c, h, w, n, d0, d1):
    """The shift form of the heads in the bf16 and fp16 conv maths against fp64 convs on
    the operands as its GEMMs round them: bf16 = RNE of every operand; fp16 = x and the head's stacked
    weight W' (both branches: one tensor, one scale) per tensor, dY per tensor for the data gradient
    (W'^T G, K = 18*C - not a multiple of 16 for C = 19 or 5), and per row of dY and x for the weight
    gradient where the plan runs the split kernel (msl_conv_wgrad_split; exact below 128 rows, C = 5).
    The only admissible difference is the fp32 accumulation (1e-5 of max|ref|)."""
    from oracle.msl_oracle import round_f16
    from maxsquareloss_amd import hip
    g = torch.Generator().manual_seed(cin + 3 * c + h)
    shape = (1, cin, n, h, w) if n > 1 else (1, cin, h, w)
    x = torch.relu(torch.randn(shape, generator=g))
    ws = [torch.randn(c, cin, 3, 3, generator=g) * 0.01 for _ in range(2)]
    bs = [torch.randn(c, generator=g) for _ in range(2)]
    gy = torch.randn((1, c) + shape[2:], generator=g) * 1e-4
    ops.set_conv_math(math)
    try:
        leaves = [t.to(DEV).requires_grad_() for t in (x, ws[0], bs[0], ws[1], bs[1])]
        y = ops.aspp2(*leaves, d0, d1, ops.PackCache())
        y.backward(gy.to(DEV))
        torch.cuda.synchronize()
    finally:
        ops.set_conv_math("fp32")
    batch = lambda t: t[0].transpose(0, 1) if n > 1 else t  # noqa: E731  [C][N][H][W] -> (N, C, H, W)
    xb, gb = batch(x).double(), batch(gy).double()
    if math == "bf16":
        rx = rd = _bf(xb)
        rws = rwd = [_bf(t) for t in ws]
        rgd = rgw = _bf(gb)
    else:
        wst = round_f16(torch.stack(ws).double())
        rx, rws, rwd, rgd = round_f16(xb), list(wst), list(wst), round_f16(gb)
        split = hip.load().msl_conv_wgrad_split(1, 1, cin, 18 * c, h, w, n)
        rd, rgw = (round_f16(xb, 1), round_f16(gb, 1)) if split else (xb, gb)
    conv = lambda a, wt, dd: F.conv2d(a, wt, padding=dd, dilation=dd)  # noqa: E731
    yr = conv(rx, rws[0], d0) + conv(rx, rws[1], d1) + (bs[0] + bs[1]).double().view(1, -1, 1, 1)
    assert _rel(batch(y.detach().cpu()), yr) < 1e-5
    xr = rx.clone().requires_grad_()
    (conv(xr, rwd[0], d0) + conv(xr, rwd[1], d1)).backward(rgd)
    assert _rel(batch(leaves[0].grad.cpu()), xr.grad) < 1e-5
    for i, (wt, dd) in enumerate(((ws[0], d0), (ws[1], d1))):
        wr = wt.double().requires_grad_()
        conv(rd, wr, dd).backward(rgw)
        assert _rel(leaves[1 + 2 * i].grad, wr.grad) < 1e-5, i
        assert _rel(leaves[2 + 2 * i].grad, gb.sum((0, 2, 3))) < 1e-5, i


@pytest.mark.parametrize("c,hi,wi,ho,wo",[(19, 65, 129, 512, 1024), (19, 33, 65, 256, 512), (16, 81, 161, 640, 1280), (3, 5, 7, 11, 13)])
def test_upsample(c, hi, wi, ho, wo):
    g = torch.Generator().manual_seed(hi)
    x = torch.randn(1, c, hi, wi, generator=g) * 3
    yr = F.interpolate(x, size=(ho, wo), mode="bilinear", align_corners=True)
    xg = x.to(DEV).requires_grad_()
    y = ops.upsample_bilinear(xg, (ho, wo))
    if wo % 16 == 0:  # torch-CPU's vectorised path (the model's shapes): bit-exact
        assert torch.equal(y.cpu(), yr), "upsample forward must be bit-exact vs torch CPU"
    else:  # torch's scalar tail rounds differently; within an ulp
        assert _rel(y, yr) < 1e-6
    gy = torch.randn(1, c, ho, wo, generator=g)
    # torch-CPU fp32 backward: same fp32 interpolation weights, different summation order
    xr = x.clone().requires_grad_()
    F.interpolate(xr, size=(ho, wo), mode="bilinear", align_corners=True).backward(gy)
    y.backward(gy.to(DEV))
    assert _rel(xg.grad, xr.grad) < 1e-5


def _softmax_ref(low, hw):
    up = F.interpolate(low, size=hw, mode="bilinear", align_corners=True)
    return up, F.softmax(up, dim=1)


@pytest.mark.parametrize("c,hi,wi,ho,wo", [(19, 33, 65, 256, 512), (16, 17, 33, 128, 256), (13, 9, 17, 64, 128)])
def test_fused_losses(c, hi, wi, ho, wo):
    g = torch.Generator().manual_seed(c)
    low = torch.randn(1, c, hi, wi, generator=g) * 4
    low2 = torch.randn(1, c, hi, wi, generator=g) * 4
    y = torch.randint(-1, c, (1, ho, wo), generator=g)
    lowg = low.to(DEV).requires_grad_()
    # --- CE
    lr = low.clone().requires_grad_()
    up, _ = _softmax_ref(lr, (ho, wo))
    ref = F.cross_entropy(up, y, ignore_index=-1)
    ref.backward()
    out = ops.ce_up(lowg, y.to(DEV).reshape(-1), (ho, wo))
    out.backward()
    assert abs(out.item() - ref.item()) <= 1e-5 * abs(ref.item())
    assert _rel(lowg.grad, lr.grad) < 1e-5
    # --- MaxSquare
    lowg.grad = None
    lr = low.clone().requires_grad_()
    _, P = _softmax_ref(lr, (ho, wo))
    ref = -torch.mean(P ** 2) / 2
    ref.backward()
    out = ops.maxsquare_up(lowg, (ho, wo))
    out.backward()
    assert abs(out.item() - ref.item()) <= 1e-5 * abs(ref.item())
    assert _rel(lowg.grad, lr.grad) < 1e-5
    # --- IW MaxSquare
    lowg.grad = None
    lr = low.clone().requires_grad_()
    _, P = _softmax_ref(lr, (ho, wo))
    maxpred, arg = torch.max(P, 1)
    hist = torch.histc(arg.float(), bins=c + 1, min=-1, max=c - 1)[1:]
    wts = 1 / torch.max(torch.pow(hist, 0.2) * torch.pow(hist.sum(), 0.8), torch.ones(1))
    ref = -torch.sum(P ** 2 * wts[arg].detach()) / c
    ref.backward()
    out, h, wv = ops.iw_maxsquare_up(lowg, (ho, wo), 0.2)
    out.backward()
    assert torch.equal(h.cpu().long(), hist.long()), "IW class histogram must be bit-exact"
    assert abs(out.item() - ref.item()) <= 1e-5 * abs(ref.item())
    assert _rel(lowg.grad, lr.grad) < 1e-5
    # --- multi-level guidance CE (gradient w.r.t. the x1 head only)
    lowg.grad = None
    lr = low.clone().requires_grad_()
    up1, P2 = _softmax_ref(lr, (ho, wo))
    _, P = _softmax_ref(low2, (ho, wo))
    m1, _ = P.max(1)
    m2, _ = P2.detach().max(1)
    pc = (P + P2.detach()) / 2
    _, ac = pc.max(1)
    lab = torch.where((m1 > 0.5) | (m2 > 0.5), ac, torch.full_like(ac, -1))
    ref = F.cross_entropy(up1, lab, ignore_index=-1)
    ref.backward()
    out = ops.multi_ce_up(lowg, low2.to(DEV), (ho, wo), 0.5)
    out.backward()
    assert abs(out.item() - ref.item()) <= 1e-5 * abs(ref.item())
    assert _rel(lowg.grad, lr.grad) < 1e-5


def test_ce_all_ignored_is_nan():
    low = torch.randn(1, 19, 9, 17, device=DEV, requires_grad=True)
    y = torch.full((64 * 128,), -1, dtype=torch.int64, device=DEV)
    out = ops.ce_up(low, y, (64, 128))
    assert torch.isnan(out).item()


def test_prob_losses():
    g = torch.Generator().manual_seed(3)
    P = torch.softmax(torch.randn(1, 19, 64, 128, generator=g) * 3, 1)
    Pr = P.clone().requires_grad_()
    ref = -torch.mean(Pr ** 2) / 2
    ref.backward()
    Pg = P.to(DEV).requires_grad_()
    out = ops.maxsquare_prob(Pg)
    out.backward()
    assert abs(out.item() - ref.item()) <= 1e-5 * abs(ref.item())
    assert _rel(Pg.grad, Pr.grad) < 1e-5
    lab = torch.randint(-1, 19, (1, 64, 128), generator=g)
    Pr = P.clone().requires_grad_()
    _, arg = torch.max(Pr, 1)
    hist = torch.histc(lab.float(), bins=20, min=-1, max=18)[1:]
    wts = 1 / torch.max(torch.pow(hist, 0.2) * torch.pow(hist.sum(), 0.8), torch.ones(1))
    ref = -torch.sum(Pr ** 2 * wts[arg]) / 19
    ref.backward()
    Pg = P.to(DEV).requires_grad_()
    out, h, _ = ops.iw_maxsquare_prob(Pg, lab.to(DEV), 0.2)
    out.backward()
    assert torch.equal(h.cpu().long(), hist.long())
    assert abs(out.item() - ref.item()) <= 1e-5 * abs(ref.item())
    assert _rel(Pg.grad, Pr.grad) < 1e-5


def test_sgd_multiplicity_matches_torch_cpu():
    from maxsquareloss_amd.utils.optim import SGD
    g = torch.Generator().manual_seed(5)
    shapes = [(64, 3, 7, 7), (256,), (19, 64, 3, 3), (10,)]
    init = [torch.randn(s, generator=g) for s in shapes]
    grads = [[torch.randn(s, generator=g) for s in shapes] for _ in range(3)]
    mult = [1, 3, 4, 1]
    # torch CPU reference: duplicated entries in group 0, last param in group 1 (10x lr)
    ref = [t.clone().requires_grad_() for t in init]
    g0 = [p for p, k in zip(ref[:3], mult[:3]) for _ in range(k)]
    opt = torch.optim.SGD([{"params": g0, "lr": 0.01}, {"params": [ref[3]], "lr": 0.1}], lr=0.01, momentum=0.9,
                          weight_decay=5e-4, foreach=False)
    mine = [t.clone().to(DEV).requires_grad_() for t in init]
    m0 = [p for p, k in zip(mine[:3], mult[:3]) for _ in range(k)]
    myopt = SGD([{"params": m0, "lr": 0.01}, {"params": [mine[3]], "lr": 0.1}], lr=0.01, momentum=0.9,
                weight_decay=5e-4)
    for step in range(3):
        for p, gr in zip(ref, grads[step]):
            p.grad = gr.clone()
        opt.step()
        myopt.zero_grad()
        for p, gr in zip(mine, grads[step]):
            # accumulate through autograd so the used-parameter hooks fire
            (p * gr.to(DEV)).sum().backward()
        myopt.step()
    torch.cuda.synchronize()
    for a, b in zip(mine, ref):
        assert _rel(a, b) < 1e-6


@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("c,h,w,res,relu,train", [(64, 129, 257, False, True, True), (256, 65, 129, True, True, True),
                                                  (1024, 33, 65, False, False, True), (64, 17, 33, True, True, False),
                                                  (512, 81, 161, False, True, True), (128, 128, 128, True, False, True),
                                                  (256, 129, 257, True, True, True)])
def test_bn_act(c, h, w, res, relu, train, fused):
    prev = ops.set_bn_fused(fused)
    try:
        _check_bn_act(c, h, w, res, relu, train)
    finally:
        ops.set_bn_fused(prev)


def _check_bn_act(c, h, w, res, relu, train):
    g = torch.Generator().manual_seed(c + h)
    x = torch.randn(1, c, h, w, generator=g) * 3 + 40.0  # large mean: the cancellation case
    r = torch.randn(1, c, h, w, generator=g) if res else None
    gamma = torch.rand(c, generator=g) + 0.5
    beta = torch.randn(c, generator=g)
    rm, rv = torch.randn(c, generator=g), torch.rand(c, generator=g) + 0.5
    gy = torch.randn(1, c, h, w, generator=g)
    bn = torch.nn.BatchNorm2d(c).to(DEV)
    with torch.no_grad():
        bn.weight.copy_(gamma)
        bn.bias.copy_(beta)
        bn.running_mean.copy_(rm)
        bn.running_var.copy_(rv)
    bn.train(train)
    xr = x.double().requires_grad_()
    gr, br = gamma.double().requires_grad_(), beta.double().requires_grad_()
    rmr, rvr = rm.double(), rv.double()
    rr = r.double().requires_grad_() if res else None
    yr = torch.nn.functional.batch_norm(xr, rmr, rvr, gr, br, train, 0.1, 1e-5)
    if res:
        yr = yr + rr
    if relu:
        yr = torch.relu(yr)
    yr.backward(gy.double())
    xg = x.to(DEV).requires_grad_()
    rg = r.to(DEV).requires_grad_() if res else None
    y = ops.bn_act(bn, xg, residual=rg, relu=relu)
    y.backward(gy.to(DEV))
    torch.cuda.synchronize()
    assert _rel(y, yr) < 1e-5
    # A pre-activation within rounding of 0 can take the other side of the ReLU (fp32 vs
    # fp64): allow a handful of such flips and compare gradients elsewhere.
    agree = torch.ones_like(yr, dtype=torch.bool)
    if relu:
        agree = (y.detach().cpu() > 0) == (yr.detach() > 0)
        assert (~agree).sum().item() <= max(2, y.numel() // 100000)
    keep = agree.double()
    assert _rel(xg.grad.cpu().double() * keep, xr.grad * keep) < 1e-4
    ch_ok = agree.view(c, -1).all(dim=1)  # channels whose sums saw no ReLU flip
    assert _rel(bn.weight.grad.cpu()[ch_ok], gr.grad[ch_ok]) < 1e-4
    assert _rel(bn.bias.grad.cpu()[ch_ok], br.grad[ch_ok]) < 1e-4
    if res:
        assert _rel(rg.grad.cpu().double() * keep, rr.grad * keep) < 1e-6
    assert _rel(bn.running_mean, rmr) < 1e-5 and _rel(bn.running_var, rvr) < 1e-5


# ----------------------------------------------------------------------------- bf16 conv math
def _bf(t):
    """The operand as the bf16 kernels see it: fp32 rounded to bf16 (RNE), exact in fp64."""
    return t.bfloat16().double()


@pytest.mark.parametrize("kind,cin,cout,h,w,d", [
    ("dconv", 256, 256, 17, 33, 2), ("dconv", 512, 512, 17, 33, 4), ("dconv", 64, 64, 33, 65, 1),
    ("pconv", 256, 1024, 17, 33, 0), ("pconv", 1024, 256, 17, 33, 0), ("aspp", 1024, 16, 17, 33, 6)])
def test_conv_bf16_math(kind, cin, cout, h, w, d):
    """BASELINE config 5's bf16 MFMA path: products of bf16-rounded operands summed in fp32.
    Reference: the same conv in fp64 on the bf16-rounded operands, so the only admissible
    difference is the fp32 accumulation (1e-5 of max|ref|, as the fp32 kernels)."""
    g = torch.Generator().manual_seed(cin + 11 * cout + d)
    k = 1 if kind == "pconv" else 3
    x = torch.randn(1, cin, h, w, generator=g)
    wt = torch.randn(cout, cin, k, k, generator=g) * 0.05
    w2 = torch.randn(cout, cin, k, k, generator=g) * 0.05
    b0, b1 = torch.randn(cout, generator=g), torch.randn(cout, generator=g)
    gy = torch.randn(1, cout, h, w, generator=g)
    ops.set_conv_math("bf16")
    try:
        xg = x.to(DEV).requires_grad_()
        wg = wt.to(DEV).requires_grad_()
        if kind == "dconv":
            y = ops.dconv3x3(xg, wg, d, ops.PackCache())
        elif kind == "pconv":
            y = ops.pconv(xg, wg, ops.PackCache(pointwise=True))
        else:
            w2g = w2.to(DEV).requires_grad_()
            y = ops.aspp2(xg, wg, b0.to(DEV), w2g, b1.to(DEV), d, 2 * d, ops.PackCache())
        y.backward(gy.to(DEV))
        torch.cuda.synchronize()
    finally:
        ops.set_conv_math("fp32")
    pad = 0 if kind == "pconv" else d
    dil = 1 if kind == "pconv" else d

    def conv(xx, ww, dd=dil, pp=pad):
        return F.conv2d(xx, ww, padding=pp, dilation=dd)

    yr = conv(_bf(x), _bf(wt))
    if kind == "aspp":
        yr = yr + conv(_bf(x), _bf(w2), 2 * d, 2 * d) + (b0 + b1).double().view(1, -1, 1, 1)
    assert _rel(y, yr) < 1e-5
    # data gradient: dy and W rounded; weight gradient: x and dy rounded
    xr = _bf(x).requires_grad_()
    conv(xr, _bf(wt)).backward(_bf(gy))
    dx_ref = xr.grad
    if kind == "aspp":
        xr2 = _bf(x).requires_grad_()
        conv(xr2, _bf(w2), 2 * d, 2 * d).backward(_bf(gy))
        dx_ref = dx_ref + xr2.grad
    wr = _bf(wt).requires_grad_()
    conv(_bf(x), wr).backward(_bf(gy))
    assert _rel(xg.grad, dx_ref) < 1e-5
    assert _rel(wg.grad, wr.grad) < 1e-5


# ----------------------------------------------------------------------------- fp16 conv math
def _f16(t):
    """The operand as the fp16 kernels see it: scaled by its tensor's power of two (absmax into
    [2^14, 2^15), dconv_kernels.h pow2_scale), rounded to fp16, unscaled - exact in fp64."""
    e = torch.frexp(t.abs().max()).exponent.item()
    sc = 2.0 ** (15 - e)
    return (t * sc).half().double() / sc


@pytest.mark.parametrize("kind,cin,cout,h,w,d", [
    ("dconv", 256, 256, 17, 33, 2), ("dconv", 512, 512, 17, 33, 4), ("dconv", 64, 64, 33, 65, 1),
    ("pconv", 256, 1024, 17, 33, 0), ("pconv", 1024, 256, 17, 33, 0), ("pconv", 256, 64, 33, 65, 0),
    ("pconv", 64, 256, 33, 65, 0)])
def test_conv_fp16_math(kind, cin, cout, h, w, d):
    """BASELINE config 5's fp16 MFMA path (msl_*_f16): products of fp16-rounded, per-tensor scaled
    operands summed in fp32 - the forward and data gradient on every M (r04: the M <= 64 GEMMs on the
    64-row fp16 tiles too), the weight gradient where both sides have >= 128 channels, exact f32 MFMA
    below.  Reference: the same conv in fp64 on the operands as
    the kernels see them, so the only admissible difference is the fp32 accumulation (1e-5 of
    max|ref|, as the fp32 kernels); operand scales far from 1 (weights 1e-2, gradients 1e-6)."""
    g = torch.Generator().manual_seed(cin + 13 * cout + d)
    k = 1 if kind == "pconv" else 3
    x = torch.relu(torch.randn(1, cin, h, w, generator=g))
    wt = torch.randn(cout, cin, k, k, generator=g) * 0.01
    gy = torch.randn(1, cout, h, w, generator=g) * 1e-6
    ops.set_conv_math("fp16")
    try:
        xg = x.to(DEV).requires_grad_()
        wg = wt.to(DEV).requires_grad_()
        if kind == "dconv":
            y = ops.dconv3x3(xg, wg, d, ops.PackCache())
        else:
            y = ops.pconv(xg, wg, ops.PackCache(pointwise=True))
        y.backward(gy.to(DEV))
        torch.cuda.synchronize()
    finally:
        ops.set_conv_math("fp32")
    pad = 0 if kind == "pconv" else d
    dil = 1 if kind == "pconv" else d
    exact = lambda t: t.double()  # noqa: E731

    def conv(xx, ww):
        return F.conv2d(xx, ww, padding=pad, dilation=dil)

    rf, rd, rw = _f16, _f16, (_f16 if min(cin, cout) >= 128 else exact)
    assert _rel(y, conv(rf(x), rf(wt))) < 1e-5
    xr = rd(x).requires_grad_()
    conv(xr, rd(wt)).backward(rd(gy))
    assert _rel(xg.grad, xr.grad) < 1e-5
    wr = rw(wt).requires_grad_()
    conv(rw(x), wr).backward(rw(gy))
    assert _rel(wg.grad, wr.grad) < 1e-5


# ----------------------------------------------------------------------------- weight packs
@pytest.mark.parametrize("kind,nb,cin,cout,for_dgrad", [
    ("d", 1, 256, 256, 0), ("d", 1, 256, 256, 1), ("d", 2, 2048, 19, 0), ("d", 2, 2048, 19, 1),
    ("d", 1, 64, 64, 0), ("d", 1, 40, 200, 1), ("d", 1, 200, 40, 0),
    ("p", 1, 1024, 256, 0), ("p", 1, 256, 1024, 1), ("p", 1, 130, 70, 0), ("p", 1, 70, 130, 1)])
def test_pack_forms_identical(kind, nb, cin, cout, for_dgrad):
    """The LDS-transposing pack+split kernel writes exactly the bytes of the element-wise pack
    followed by k_split_pack (fp32 pack and bf16x6 planes), incl. padding rows and 2 branches."""
    from maxsquareloss_amd import hip
    lib = hip.load()
    k = 3 if kind == "d" else 1
    w = torch.randn(nb, cout, cin, k, k, generator=torch.Generator().manual_seed(cin * 7 + cout)).to(DEV)
    total = lib.msl_dconv_packed_elems(nb, cin, cout, for_dgrad) if kind == "d" else \
        lib.msl_pconv_packed_elems(cin, cout, for_dgrad)
    bufs = []
    for form in (0, 1):
        fm = hip.Forms(hip.FORMS.f32_form, 1, form, 1)  # the call's own forms (ABI 3), not the process's
        buf = torch.full((total,), float("nan"), device=DEV)
        if kind == "d":
            st = lib.msl_dconv_pack(w.data_ptr(), cout * cin * 9, nb, cin, cout, for_dgrad, buf.data_ptr(),
                                    ctypes.addressof(fm), hip.stream_ptr())
        else:
            st = lib.msl_pconv_pack(w.data_ptr(), cin, cout, for_dgrad, buf.data_ptr(), ctypes.addressof(fm),
                                    hip.stream_ptr())
        assert st == 0
        bufs.append(buf)
    torch.cuda.synchronize()
    assert torch.equal(bufs[0].view(torch.int32), bufs[1].view(torch.int32))


def _defined(buf, form):
    """The defined part of a packed buffer (fp32 pack F, planes region 1.5 F, 320-float tail): the
    bf16x6 planes fill their region; the f16x3 ones its first F floats, and that form writes the
    weights' absmax partials (256) and {scale, 1/scale} into the tail."""
    f32 = (buf.numel() - 320) * 2 // 5
    if form != "f16x3":
        return buf[:buf.numel() - 320].view(torch.int32)
    return torch.cat([buf[:2 * f32], buf[buf.numel() - 320:buf.numel() - 62]]).view(torch.int32)


def test_pack_batch_matches_per_conv_packs(f32_form):
    """ops.PackBatch (msl_conv_pack_many: every pack of a step in one launch per tap count) writes
    exactly the bytes of the per-conv msl_*_pack calls, for 9- and 1-tap packs, both directions,
    a 2-branch ASPP pack and M <= 64 (no planes, except in f16x3) - exactly the stale ones - in every
    fp32 form (f16x3: the fp16 planes and the weights' scale too)."""
    import torch.nn as nn
    g = torch.Generator().manual_seed(5)

    class Holder(nn.Module):
        def __init__(self, weights, cin, cout, pointwise):
            super().__init__()
            self.ws = nn.ParameterList([nn.Parameter(w) for w in weights])
            self._pack = ops.PackCache(pointwise=pointwise)
            self.dims = (cin, cout)

        def use(self):
            cin, cout = self.dims
            for d in (0, 1):
                self._pack.get(list(self.ws), cin, cout, d)

    specs = [([torch.randn(256, 256, 3, 3, generator=g)], 256, 256, False),
             ([torch.randn(64, 40, 3, 3, generator=g)], 40, 64, False),
             (list(torch.randn(2, 19, 1024, 3, 3, generator=g).unbind(0)), 1024, 19, False),
             ([torch.randn(1024, 256, 1, 1, generator=g)], 256, 1024, True),
             ([torch.randn(70, 130, 1, 1, generator=g)], 130, 70, True)]
    hs = nn.ModuleList([Holder(*s) for s in specs]).to(DEV)
    for h in hs:  # the 2-branch pack reads branch 1 at a fixed stride from branch 0: one storage
        if len(h.ws) == 2:
            both = torch.stack([h.ws[0].data, h.ws[1].data])
            h.ws[0].data, h.ws[1].data = both[0], both[1]
    for h in hs:
        h.use()  # lazy packs; marks both directions used
    batch = ops.PackBatch(hs)
    assert len(batch.caches) == len(specs)
    with torch.no_grad():
        for h in hs:
            for w in h.ws:
                w.mul_(-1.5)
    for h in hs:
        h.use()  # lazy repack of the new weights
    torch.cuda.synchronize()
    ref = [{d: h._pack.buf[d].clone() for d in (0, 1)} for h in hs]
    assert not batch.run()  # nothing stale: no launch
    with torch.no_grad():
        hs[0].ws[0].mul_(1.0)  # one stale conv (same values): only its two packs are redone
        for d in (0, 1):
            hs[0]._pack.buf[d].fill_(float("nan"))
    assert batch.run() and batch.launches == 1
    torch.cuda.synchronize()
    for d in (0, 1):
        assert torch.equal(_defined(hs[0]._pack.buf[d], f32_form), _defined(ref[0][d], f32_form))
    with torch.no_grad():
        for h in hs:
            for w in h.ws:
                w.mul_(-2.0)
            for d in (0, 1):
                h._pack.buf[d].fill_(float("nan"))
    assert batch.run() and batch.launches == 2
    with torch.no_grad():
        for h in hs:
            for w in h.ws:
                w.mul_(-0.5)  # back to the values of the reference packs (x(-2)x(-0.5) = 1)
            for d in (0, 1):
                h._pack.buf[d].fill_(float("nan"))
    assert batch.run() and batch.launches == 3
    torch.cuda.synchronize()
    for h, r in zip(hs, ref):
        for d in (0, 1):
            total = ops.hip.load().msl_dconv_packed_elems(len(h.ws), h.dims[0], h.dims[1], d) if not h._pack.pointwise \
                else ops.hip.load().msl_pconv_packed_elems(h.dims[0], h.dims[1], d)
            m = h.dims[1] if d == 0 else h.dims[0]
            # M <= 64: no planes (and no tail) behind the fp32 pack, except in the f16x3 form, which
            # splits every M since r03 (the <= 64-row 3x3 / ASPP GEMMs run f16x3 on 64-row tiles)
            n = (total - 320) * 2 // 5
            planes = m > 64 or f32_form == "f16x3"
            if planes:
                assert torch.equal(_defined(h._pack.buf[d], f32_form), _defined(r[d], f32_form)), (h.dims, d)
            else:
                assert torch.equal(h._pack.buf[d][:n].view(torch.int32), r[d][:n].view(torch.int32)), (h.dims, d)
                # the per-conv calls never touch the planes region of such a pack; neither does the batch
                assert torch.isnan(h._pack.buf[d][n:]).all()
            # lazy get() finds them fresh: no repack
            key = h._pack.key[d]
            h._pack.get(list(h.ws), h.dims[0], h.dims[1], d)
            assert h._pack.key[d] == key


@pytest.mark.parametrize("cin,cout,h,w", [(1024, 256, 17, 33), (2048, 512, 9, 17), (256, 1024, 17, 33),
                                           (256, 64, 33, 65), (512, 128, 17, 33), (1024, 256, 65, 129)])
def test_pconv_dgrad_accumulate(cin, cout, h, w, f32_form):
    """msl_pconv_dgrad_acc: dx += W^T dy in the GEMM's own epilogue / piece reduce."""
    from maxsquareloss_amd import hip
    lib = hip.load()
    g = torch.Generator().manual_seed(cin + cout)
    p = h * w
    wt = torch.randn(cout, cin, 1, 1, generator=g) * 0.05
    gy = torch.randn(1, cout, h, w, generator=g)
    dx0 = torch.randn(1, cin, h, w, generator=g)
    ref = dx0.double() + torch.mm(wt.view(cout, cin).double().t(), gy.view(cout, p).double()).view(1, cin, h, w)
    cache = ops.PackCache(pointwise=True)
    wd = wt.to(DEV)
    packed_d = cache.get([wd], cin, cout, 1)
    dx = dx0.to(DEV)
    wsb = lib.msl_pconv_dgrad_workspace(cin, cout, p)
    ws = hip.workspace(wsb, dx.device)
    assert lib.msl_pconv_dgrad_acc(gy.to(DEV).data_ptr(), packed_d.data_ptr(), dx.data_ptr(), cin, cout, p, 1,
                                   hip.forms(), ws.data_ptr(), wsb, hip.stream_ptr()) == 0
    torch.cuda.synchronize()
    assert _rel(dx, ref) < 1e-5


@pytest.mark.parametrize("kind", ["identity", "downsample", "downsample_s2"])
def test_bottleneck_fused_residual_grad(f32_form, monkeypatch, kind):
    """Bottleneck with an identity residual: the residual's gradient summed into x's gradient by
    conv1's data-gradient GEMM (ops.ResidualGrad) equals autograd's separate accumulation; r05: likewise
    a block with a downsample conv (layer1.0 / layer3.0, and layer2.0's stride 2), whose data gradient
    conv1's GEMM sums instead of autograd."""
    from torch import nn
    from maxsquareloss_amd.graphs.models import deeplab_multi as dm
    torch.manual_seed(3)
    if kind == "identity":
        blk, cin, cout, hw, ho = dm.Bottleneck(1024, 256, dilation=2), 1024, 1024, (17, 33), (17, 33)
    else:
        s = 2 if kind == "downsample_s2" else 1
        ds = nn.Sequential(dm.conv1x1(512, 1024, s), nn.BatchNorm2d(1024, affine=dm.affine_par))
        blk, cin, cout = dm.Bottleneck(512, 256, stride=s, dilation=1, downsample=ds), 512, 1024
        hw = (33, 65) if s == 2 else (17, 33)
        ho = ((hw[0] + 1) // 2, (hw[1] + 1) // 2) if s == 2 else hw
    blk = blk.to(DEV).train()
    x = (torch.randn(1, cin, *hw) * 2).to(DEV)
    gy = torch.randn(1, cout, *ho).to(DEV)
    out = {}
    for fused in (True, False):
        monkeypatch.setattr(dm, "FUSE_RESIDUAL_GRAD", fused)
        xg = x.clone().requires_grad_()
        for prm in blk.parameters():
            prm.grad = None
        y = blk(xg)
        y.backward(gy)
        torch.cuda.synchronize()
        out[fused] = (y.detach().clone(), xg.grad.clone(), [prm.grad.clone() for prm in blk.parameters()])
    assert torch.equal(out[True][0], out[False][0])
    assert _rel(out[True][1], out[False][1].double()) < 1e-6
    for a, b in zip(out[True][2], out[False][2]):
        assert _rel(a, b.double()) < 1e-6


@pytest.mark.parametrize("nimg", [1, 2])
@pytest.mark.parametrize("math", ["fp32", "fp16", "bf16"])
def test_masked_residual_grad(monkeypatch, math, nimg):
    """r06: an identity block's residual gradient left unmaterialised (ops.MaskedResidual, the ReLU mask
    applied in conv1's data-gradient epilogue, msl_pconv_dgrad_resmask) gives bit-identical gradients to
    bn3 writing it (RESMASK_DGRAD off); bf16, whose form has no epilogue, materialises it."""
    from maxsquareloss_amd.graphs.models import deeplab_multi as dm
    made = []

    class Counted(ops.MaskedResidual):
        __slots__ = ()

        def __init__(self, *a):
            super().__init__(*a)
            made.append(1)

    monkeypatch.setattr(ops, "MaskedResidual", Counted)
    torch.manual_seed(5 + nimg)
    blk = dm.Bottleneck(1024, 256, dilation=2).to(DEV).train()
    shape = (1, 1024, nimg, 17, 33) if nimg > 1 else (1, 1024, 17, 33)
    x = (torch.randn(*shape) * 2).to(DEV)
    gy = torch.randn(*shape).to(DEV)
    out = {}
    prev = ops.CONV_MATH
    try:
        ops.set_conv_math(math)
        for lazy in (True, False):
            monkeypatch.setattr(ops, "RESMASK_DGRAD", lazy)
            xg = x.clone().requires_grad_()
            for prm in blk.parameters():
                prm.grad = None
            y = blk(xg)
            y.backward(gy)
            torch.cuda.synchronize()
            out[lazy] = (y.detach().clone(), xg.grad.clone(), [prm.grad.clone() for prm in blk.parameters()])
    finally:
        ops.set_conv_math(prev)
    assert len(made) == (1 if math != "bf16" else 0)
    assert torch.equal(out[True][0], out[False][0])
    assert torch.equal(out[True][1], out[False][1])
    for a, b in zip(out[True][2], out[False][2]):
        assert torch.equal(a, b)


@pytest.mark.parametrize("nimg", [1, 2])
def test_masked_residual_materialize(nimg):
    """MaskedResidual.materialize (the bf16 path) equals dy * (y > 0) of the BN's own forward."""
    torch.manual_seed(9)
    bn = torch.nn.BatchNorm2d(256).to(DEV).train()
    shape = (1, 256, nimg, 17, 33) if nimg > 1 else (1, 256, 17, 33)
    x = torch.randn(*shape).to(DEV).requires_grad_()
    res = torch.randn(*shape).to(DEV)
    hold = ops.ResidualGrad()
    y = ops.bn_act(bn, x, residual=res, relu=True, residual_grad=hold)
    gy = torch.randn(*shape).to(DEV)
    y.backward(gy)
    torch.cuda.synchronize()
    assert isinstance(hold.g, ops.MaskedResidual)
    assert torch.equal(hold.g.materialize(), torch.where(y > 0, gy, torch.zeros_like(gy)))


@pytest.mark.parametrize("cin,cout,h,w", [(256, 1024, 65, 129), (512, 2048, 64, 128), (2048, 512, 65, 129),
                                           (1024, 2048, 17, 33)])
def test_sk_hybrid_schedule(cin, cout, h, w, f32_form):
    """Forward-form schedule: data-parallel rounds + a stream-K remainder (default; 528 / 1056
    tiles leave 16 / 32 split tiles, 2048 x 8192 is exactly 1024 whole tiles and launches no
    reduce) and pure stream-K (msl_forms.sk_hybrid 0) both match fp64, forward and data
    gradient."""
    from maxsquareloss_amd import hip
    g = torch.Generator().manual_seed(cin + 11 * cout)
    x = torch.randn(1, cin, h, w, generator=g)
    wt = torch.randn(cout, cin, 1, 1, generator=g) * 0.05
    gy = torch.randn(1, cout, h, w, generator=g)
    xr, wr = x.double().requires_grad_(), wt.double().requires_grad_()
    yr = F.conv2d(xr, wr)
    yr.backward(gy.double())
    outs = []
    try:
        for hybrid in (1, 0):
            hip.set_form("sk_hybrid", hybrid)
            xg = x.to(DEV).requires_grad_()
            wg = wt.to(DEV).requires_grad_()
            y = ops.pconv(xg, wg, ops.PackCache(pointwise=True))
            y.backward(gy.to(DEV))
            torch.cuda.synchronize()
            assert _rel(y, yr) < 1e-5, hybrid
            assert _rel(xg.grad, xr.grad) < 1e-5, hybrid
            outs.append((y.detach(), xg.grad))
    finally:
        hip.set_form("sk_hybrid", 1)
    # the two schedules differ only in the fp32 summation order of split tiles
    assert _rel(outs[0][0], outs[1][0].double()) < 4e-6
    assert _rel(outs[0][1], outs[1][1].double()) < 4e-6
    with pytest.raises(hip.MSLError):
        hip.set_form("sk_hybrid", 2)


@pytest.mark.parametrize("cin,cout,h,w", [(256, 1024, 65, 129), (512, 2048, 17, 33), (128, 512, 33, 65),
                                           (1024, 256, 65, 129), (200, 328, 9, 31)])
@pytest.mark.parametrize("form", ["bf16x6", "f16x3"])
def test_pconv_wgrad_accumulate_both_orientations(cin, cout, h, w, form):
    """msl_pconv_wgrad, accumulate = 1, in both split forms: with cout > cin the kernel runs on the
    swapped operands (the image pre-split, dW^T tiles transposed by the reduce); either way
    dW += dy x^T.  f16x3: msl_pconv_wgrad_sc given the operands' per-row absmax partials
    (msl_absmax_partials) writes exactly the bytes of the plain call, which reduces them itself."""
    from maxsquareloss_amd import hip
    lib = hip.load()
    prev = ops.set_f32_form(form)
    try:
        g = torch.Generator().manual_seed(cin * 5 + cout)
        p = h * w
        x = torch.randn(cin, p, generator=g)
        gy = torch.randn(cout, p, generator=g)
        dw0 = torch.randn(cout, cin, generator=g)
        ref = dw0.double() + gy.double() @ x.double().t()
        xd, gd, dw = x.to(DEV), gy.to(DEV), dw0.to(DEV)
        wsb = lib.msl_pconv_wgrad_workspace(cin, cout, p)
        ws = hip.workspace(wsb, xd.device)
        assert lib.msl_pconv_wgrad(xd.data_ptr(), gd.data_ptr(), dw.data_ptr(), cin, cout, p, 1, hip.forms(),
                                   ws.data_ptr(), wsb, hip.stream_ptr()) == 0
        torch.cuda.synchronize()
        assert _rel(dw, ref) < 1e-5
        if form == "f16x3":
            xp, gp = torch.empty(cin, device=DEV), torch.empty(cout, device=DEV)
            for t, q, rows in ((xd, xp, cin), (gd, gp, cout)):
                assert lib.msl_absmax_partials(t.data_ptr(), rows, p, q.data_ptr(), hip.stream_ptr()) == 0
            assert torch.equal(xp.cpu(), x.abs().amax(1)) and torch.equal(gp.cpu(), gy.abs().amax(1))  # per row
            dw2 = dw0.to(DEV)
            assert lib.msl_pconv_wgrad_sc(xd.data_ptr(), gd.data_ptr(), dw2.data_ptr(), cin, cout, p, 1, hip.forms(),
                                          ws.data_ptr(), wsb, hip.stream_ptr(), xp.data_ptr(), cin, gp.data_ptr(), cout) == 0
            torch.cuda.synchronize()
            assert torch.equal(dw2, dw)
    finally:
        ops.set_f32_form(prev)


def _elem_err(out, ref, bound):
    """max over elements of |out - ref| / (the same conv of |operands|): the error relative to the
    element's own sum of |terms|, the measure fp32 accumulation is judged by."""
    out, ref, bound = (t.detach().double().cpu() for t in (out, ref, bound))
    return ((out - ref).abs() / bound.clamp_min(1e-300)).max().item()


@pytest.mark.gpu
@pytest.mark.parametrize("xs,gs", [(1.0, 1.0), (1e-20, 1e15), (3e4, 1e-30)])
@pytest.mark.parametrize("cin,cout,h,w,d", [(256, 256, 33, 65, 2), (512, 512, 17, 33, 4)])
def test_f16x3_is_fp32_accurate(cin, cout, h, w, d, xs, gs):
    """The f16x3 form (per-tensor power-of-two scale, two fp16 terms, three fp16 MFMAs) against fp64,
    per element relative to the element's sum of |terms|, next to the exact fp32 MFMA and bf16x6 on
    the same operands: fwd, data and weight gradients, at unit scale and at operand scales far
    outside fp16's range (weights ~1e-2, the 1e-20 / 1e-30 / 3e4 / 1e15 factors exercise the
    scaling).  Bar: within 2x the exact fp32 MFMA's error, and below 2e-7."""
    g = torch.Generator().manual_seed(cin + h)
    x = torch.relu(torch.randn(1, cin, h, w, generator=g)) * xs
    wt = torch.randn(cout, cin, 3, 3, generator=g) * 0.01
    gy = torch.randn(1, cout, h, w, generator=g) * gs
    xr, wr = x.double().requires_grad_(), wt.double().requires_grad_()
    yr = F.conv2d(xr, wr, padding=d, dilation=d)
    yr.backward(gy.double())
    # sums of |terms| of every output element (conv of the absolute operands)
    xa, wa, ga = x.double().abs().requires_grad_(), wt.double().abs().requires_grad_(), gy.double().abs()
    ya = F.conv2d(xa, wa, padding=d, dilation=d)
    ya.backward(ga)
    errs = {}
    for form in ("mfma_f32", "bf16x6", "f16x3"):
        prev = ops.set_f32_form(form)
        try:
            xg = x.to(DEV).requires_grad_()
            wg = wt.to(DEV).requires_grad_()
            y = ops.dconv3x3(xg, wg, d, ops.PackCache())
            y.backward(gy.to(DEV))
            torch.cuda.synchronize()
            errs[form] = (_elem_err(y, yr, ya), _elem_err(xg.grad, xr.grad, xa.grad),
                          _elem_err(wg.grad, wr.grad, wa.grad))
        finally:
            ops.set_f32_form(prev)
    for i, what in enumerate(("fwd", "dgrad", "wgrad")):
        e, ref = errs["f16x3"][i], errs["mfma_f32"][i]
        assert e < 2e-7 and e <= 2.0 * max(ref, 1e-8), (what, errs)


@pytest.mark.gpu
@pytest.mark.parametrize("kind,cin,cout,h,w", [("3x3", 256, 256, 33, 65), ("1x1", 256, 1024, 33, 65),
                                               ("1x1", 1024, 256, 33, 65), ("3x3", 512, 512, 17, 33)])
def test_f16x3_channel_spread_accuracy(kind, cin, cout, h, w):
    """with one power-of-two scale per tensor, a channel far below the tensor's absolute
    maximum loses its lo term to fp16 subnormals.  Here every channel of x and of dy gets its own
    scale, log-uniform over 1e-8 .. 1 (per-channel spread within one tensor), and each output
    element's error against fp64, relative to its own sum of |terms|, must stay within 2x the exact
    fp32 MFMA's (and below 1e-6) - forward, data and weight gradients (the 1x1 shapes include the
    swapped-operand weight gradient, cout > cin).  The weight gradient's output rows / columns ARE
    the channels, so it scales every row of dY and of x by its own power of two (rowscale); the
    forward and data gradient sum over channels, where a tiny channel's terms are tiny in the
    element's sum too."""
    g = torch.Generator().manual_seed(cin * 5 + cout + h)
    k = 3 if kind == "3x3" else 1
    d = 2 if k == 3 else 0
    cs = 10.0 ** (-8.0 * torch.rand(cin, generator=g))
    gsc = 10.0 ** (-8.0 * torch.rand(cout, generator=g))
    x = torch.relu(torch.randn(1, cin, h, w, generator=g)) * cs.view(1, cin, 1, 1)
    wt = torch.randn(cout, cin, k, k, generator=g) * 0.01
    gy = torch.randn(1, cout, h, w, generator=g) * gsc.view(1, cout, 1, 1)
    conv = (lambda a, b: F.conv2d(a, b, padding=d, dilation=d)) if k == 3 else (lambda a, b: F.conv2d(a, b))
    xr, wr = x.double().requires_grad_(), wt.double().requires_grad_()
    conv(xr, wr).backward(gy.double())
    xa, wa = x.double().abs().requires_grad_(), wt.double().abs().requires_grad_()
    ya = conv(xa, wa)
    ya.backward(gy.double().abs())
    yr = conv(x.double(), wt.double())
    errs = {}
    for form in ("mfma_f32", "f16x3"):
        prev = ops.set_f32_form(form)
        try:
            xg, wg = x.to(DEV).requires_grad_(), wt.to(DEV).requires_grad_()
            y = (ops.dconv3x3(xg, wg, d, ops.PackCache()) if k == 3 else
                 ops.pconv(xg, wg, ops.PackCache(pointwise=True)))
            y.backward(gy.to(DEV))
            torch.cuda.synchronize()
            errs[form] = (_elem_err(y, yr, ya), _elem_err(xg.grad, xr.grad, xa.grad),
                          _elem_err(wg.grad, wr.grad, wa.grad))
        finally:
            ops.set_f32_form(prev)
    for i, what in enumerate(("fwd", "dgrad", "wgrad")):
        e, ref = errs["f16x3"][i], errs["mfma_f32"][i]
        assert e < 1e-6 and e <= 2.0 * max(ref, 1e-8), (what, errs)


@pytest.mark.gpu
@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("c,h,w,res,relu", [(256, 65, 129, True, True), (64, 129, 257, False, True),
                                             (1024, 33, 65, False, False)])
def test_bn_absmax_outputs(c, h, w, res, relu, fused):
    """msl_bn_fwd_am / msl_bn_bwd_am: the same y / dx / dres / dgamma / dbeta bytes as msl_bn_fwd /
    msl_bn_bwd, plus absmax[c] = max |y[c]| (forward) and max |dx[c]| (backward) exactly, in the
    fused and the split kernel forms (the f16x3 convs' operand partials)."""
    from maxsquareloss_amd import hip
    lib = hip.load()
    prev = ops.set_bn_fused(fused)
    try:
        g = torch.Generator().manual_seed(c * 3 + h)
        p = h * w
        x = (torch.randn(c, p, generator=g) * 3 + 1).to(DEV)
        r = torch.randn(c, p, generator=g).to(DEV) if res else None
        gamma = (torch.rand(c, generator=g) + 0.5).to(DEV)
        beta = torch.randn(c, generator=g).to(DEV)
        gy = torch.randn(c, p, generator=g).to(DEV)
        wsb = lib.msl_bn_workspace(c, p, 1)
        ws = hip.workspace(wsb, x.device)
        s = hip.stream_ptr()
        outs = []
        for am in (False, True):
            rm, rv = torch.zeros(c, device=DEV), torch.ones(c, device=DEV)
            y, sm, si = torch.empty_like(x), torch.empty(c, device=DEV), torch.empty(c, device=DEV)
            dx, dres = torch.empty_like(x), torch.empty_like(x)
            dg, db = torch.empty(c, device=DEV), torch.empty(c, device=DEV)
            fa, ba = torch.full((c,), -1.0, device=DEV), torch.full((c,), -1.0, device=DEV)
            fargs = (x.data_ptr(), gamma.data_ptr(), beta.data_ptr(), hip.ptr(r), y.data_ptr(), rm.data_ptr(),
                     rv.data_ptr(), None, sm.data_ptr(), si.data_ptr(), c, p, 1, 1, 1, 0.1, 1e-5, int(relu), hip.forms(),
                     ws.data_ptr(), wsb, s)
            bargs = (gy.data_ptr(), x.data_ptr(), y.data_ptr(), gamma.data_ptr(), sm.data_ptr(), si.data_ptr(),
                     dx.data_ptr(), dres.data_ptr(), dg.data_ptr(), db.data_ptr(), c, p, 1, 1, int(relu), 0, hip.forms(),
                     ws.data_ptr(), wsb, s)
            if am:
                assert lib.msl_bn_fwd_am(*fargs, fa.data_ptr()) == 0
                assert lib.msl_bn_bwd_am(*bargs, ba.data_ptr()) == 0
            else:
                assert lib.msl_bn_fwd(*fargs) == 0
                assert lib.msl_bn_bwd(*bargs) == 0
            torch.cuda.synchronize()
            outs.append((y, dx, dres, dg, db, fa, ba))
        for a, b in zip(outs[0][:5], outs[1][:5]):
            assert torch.equal(a, b)
        y, dx, _, _, _, fa, ba = outs[1]
        assert torch.equal(fa, y.abs().amax(dim=1))
        assert torch.equal(ba, dx.abs().amax(dim=1))
    finally:
        ops.set_bn_fused(prev)


@pytest.mark.gpu
@pytest.mark.parametrize("training", [1, 0])
@pytest.mark.parametrize("c,h,w,nimg", [(64, 161, 321, 2), (256, 33, 65, 2), (3, 7, 5, 3)])
def test_bn_absmax_split_forms_images(c, h, w, nimg, training):
    """The split BN kernels' absmax (r05: folded into the flat apply kernels, zeroed by the stats /
    reduce launch or, in eval mode, by a zeroing launch): max |y| / |dx| over every image of the
    channel ([C][NI][P]), blocks that cross rows and channels included, exactly; stale values in the
    output buffer are overwritten."""
    from maxsquareloss_amd import hip
    lib = hip.load()
    prev = ops.set_bn_fused(False)
    try:
        g = torch.Generator().manual_seed(c + h + nimg)
        p = h * w
        x = (torch.randn(c, nimg, p, generator=g) * 3 + 1).to(DEV)
        gamma = (torch.rand(c, generator=g) + 0.5).to(DEV)
        beta = torch.randn(c, generator=g).to(DEV)
        gy = torch.randn(c, nimg, p, generator=g).to(DEV)
        wsb = lib.msl_bn_workspace(c, p, nimg)
        ws = hip.workspace(wsb, x.device)
        s = hip.stream_ptr()
        rm, rv = torch.randn(c, generator=g).to(DEV), (torch.rand(c, generator=g) + 0.5).to(DEV)
        y, sm, si = torch.empty_like(x), torch.empty(c * nimg, device=DEV), torch.empty(c * nimg, device=DEV)
        dx = torch.empty_like(x)
        dg, db = torch.empty(c, device=DEV), torch.empty(c, device=DEV)
        fa, ba = torch.full((c,), 1e30, device=DEV), torch.full((c,), 1e30, device=DEV)  # stale
        assert lib.msl_bn_fwd_am(x.data_ptr(), gamma.data_ptr(), beta.data_ptr(), None, y.data_ptr(), rm.data_ptr(),
                                 rv.data_ptr(), None, sm.data_ptr(), si.data_ptr(), c, p, nimg, training, 0, 0.1,
                                 1e-5, 0, hip.forms(), ws.data_ptr(), wsb, s, fa.data_ptr()) == 0
        assert lib.msl_bn_bwd_am(gy.data_ptr(), x.data_ptr(), y.data_ptr(), gamma.data_ptr(), sm.data_ptr(),
                                 si.data_ptr(), dx.data_ptr(), None, dg.data_ptr(), db.data_ptr(), c, p, nimg,
                                 training, 0, 0, hip.forms(), ws.data_ptr(), wsb, s, ba.data_ptr()) == 0
        torch.cuda.synchronize()
        assert torch.equal(fa, y.abs().reshape(c, -1).amax(dim=1))
        assert torch.equal(ba, dx.abs().reshape(c, -1).amax(dim=1))
    finally:
        ops.set_bn_fused(prev)


@pytest.mark.gpu
@pytest.mark.parametrize("c,h,w,nimg", [(256, 65, 129, 2), (512, 65, 129, 1), (128, 33, 65, 2), (2048, 17, 33, 2)])
def test_bn_bwd_relu_mask_recompute(c, h, w, nimg):
    """msl_bn_bwd_am_beta with y = NULL (the fused kernel recomputes the ReLU mask from x, beta and the
    saved statistics): the same dx / dgamma / dbeta / absmax bytes as msl_bn_bwd_am reading y, incl.
    pre-activations that are exactly 0 (x = mean, beta = 0 channels); y = NULL is refused where the
    split kernels would run, and by msl_bn_bwd_am."""
    from maxsquareloss_amd import hip
    lib = hip.load()
    prev = ops.set_bn_fused(True)
    try:
        g = torch.Generator().manual_seed(c + nimg)
        p = h * w
        x = torch.randn(c, nimg, p, generator=g) * 3 + 1
        x[:, :, : p // 2] = x[:, :, :1]  # half of each row equal: many pre-activations at the mean
        x = x.reshape(c, nimg * p).to(DEV)
        gamma = (torch.rand(c, generator=g) + 0.5).to(DEV)
        beta = torch.randn(c, generator=g)
        beta[::3] = 0.0
        beta = beta.to(DEV)
        gy = torch.randn(c, nimg * p, generator=g).to(DEV)
        wsb = lib.msl_bn_workspace(c, p, nimg)
        ws = hip.workspace(wsb, x.device)
        s = hip.stream_ptr()
        rm, rv = torch.zeros(c, device=DEV), torch.ones(c, device=DEV)
        y = torch.empty_like(x)
        sm, si = torch.empty(c * nimg, device=DEV), torch.empty(c * nimg, device=DEV)
        assert lib.msl_bn_fwd(x.data_ptr(), gamma.data_ptr(), beta.data_ptr(), None, y.data_ptr(), rm.data_ptr(),
                              rv.data_ptr(), None, sm.data_ptr(), si.data_ptr(), c, p, nimg, 1, 1, 0.1, 1e-5, 1,
                              hip.forms(), ws.data_ptr(), wsb, s) == 0
        assert lib.msl_bn_uses_fused(c, p, 1, hip.forms()) == 1
        outs = []
        for remask in (False, True):
            dx = torch.empty_like(x)
            dg, db, am = (torch.empty(c, device=DEV) for _ in range(3))
            args = (gy.data_ptr(), x.data_ptr(), None if remask else y.data_ptr(), gamma.data_ptr(), beta.data_ptr(),
                    sm.data_ptr(), si.data_ptr(), dx.data_ptr(), None, dg.data_ptr(), db.data_ptr(), c, p, nimg, 1, 1, 0,
                    hip.forms(), ws.data_ptr(), wsb, s, am.data_ptr())
            assert lib.msl_bn_bwd_am_beta(*args) == 0
            torch.cuda.synchronize()
            outs.append((dx, dg, db, am))
        assert (y == 0).float().mean().item() > 0.2  # the mask matters
        for a, b in zip(*outs):
            assert torch.equal(a, b)
        # refusals: the split forms read y; msl_bn_bwd_am always needs it
        assert lib.msl_bn_bwd_am(gy.data_ptr(), x.data_ptr(), None, gamma.data_ptr(), sm.data_ptr(), si.data_ptr(),
                                 dx.data_ptr(), None, dg.data_ptr(), db.data_ptr(), c, p, nimg, 1, 1, 0, hip.forms(),
                                 ws.data_ptr(), wsb, s, None) == -3
        big = 129 * 257  # fused, but the 33-element form keeps reading y (checked before any launch)
        assert lib.msl_bn_uses_fused(256, big, 1, hip.forms()) == 1
        assert lib.msl_bn_bwd_am_beta(gy.data_ptr(), x.data_ptr(), None, gamma.data_ptr(), beta.data_ptr(),
                                      sm.data_ptr(), si.data_ptr(), dx.data_ptr(), None, dg.data_ptr(), db.data_ptr(),
                                      256, big, 1, 1, 1, 0, hip.forms(), ws.data_ptr(), lib.msl_bn_workspace(256, big, 1), s,
                                      None) == -3
        ops.set_bn_fused(False)
        assert lib.msl_bn_bwd_am_beta(gy.data_ptr(), x.data_ptr(), None, gamma.data_ptr(), beta.data_ptr(),
                                      sm.data_ptr(), si.data_ptr(), dx.data_ptr(), None, dg.data_ptr(), db.data_ptr(),
                                      c, p, nimg, 1, 1, 0, hip.forms(), ws.data_ptr(), wsb, s, None) == -3
    finally:
        ops.set_bn_fused(prev)


@pytest.mark.gpu
@pytest.mark.parametrize("c,h,w,nimg", [(1024, 65, 129, 2), (256, 129, 257, 2), (512, 65, 129, 1), (2048, 17, 33, 2)])
def test_bn_relu_mask_bits(c, h, w, nimg):
    """msl_bn_fwd_mask / msl_bn_bwd_mask (r05): the residual BN + ReLU writes y > 0 as bits (bit e % 64 of
    word [row][e / 64]) and its backward reads them instead of y - the same y / statistics / dx / dres /
    dgamma / dbeta / absmax bytes as msl_bn_fwd_am + msl_bn_bwd_am_beta reading y, incl. pre-activations
    that are exactly 0, the 33-element form (layer1's 33153 px) and a tail word; refused without relu or
    under the split kernels."""
    from maxsquareloss_amd import hip
    lib = hip.load()
    g = torch.Generator().manual_seed(c + 7 * nimg)
    p = h * w
    x = torch.randn(c, nimg, p, generator=g) * 3 + 1
    x[:, :, : p // 3] = x[:, :, :1]  # a third of each row at the mean: pre-activation = beta + residual
    x = x.reshape(c, nimg * p).to(DEV)
    res = torch.randn(c, nimg * p, generator=g)
    res[::2, : p // 3] = 0.0
    res = res.to(DEV)
    gamma = (torch.rand(c, generator=g) + 0.5).to(DEV)
    beta = torch.randn(c, generator=g)
    beta[::2] = 0.0
    beta = beta.to(DEV)
    gy = torch.randn(c, nimg * p, generator=g).to(DEV)
    wsb = lib.msl_bn_workspace(c, p, nimg)
    ws = hip.workspace(wsb, x.device)
    s = hip.stream_ptr()
    nw = (p + 63) // 64
    assert lib.msl_bn_relu_mask_bytes(c, p, nimg) == c * nimg * nw * 8
    assert lib.msl_bn_uses_fused(c, p, 1, hip.forms()) == 1
    outs = []
    for use_bits in (False, True):
        rm, rv = torch.zeros(c, device=DEV), torch.ones(c, device=DEV)
        y = torch.empty_like(x)
        sm, si = torch.empty(c * nimg, device=DEV), torch.empty(c * nimg, device=DEV)
        fa, ba = torch.empty(c, device=DEV), torch.empty(c, device=DEV)
        bits = torch.full((c * nimg * nw,), -1, dtype=torch.int64, device=DEV)
        fargs = (x.data_ptr(), gamma.data_ptr(), beta.data_ptr(), res.data_ptr(), y.data_ptr(), rm.data_ptr(),
                 rv.data_ptr(), None, sm.data_ptr(), si.data_ptr(), c, p, nimg, 1, 1, 0.1, 1e-5, 1, hip.forms(),
                 ws.data_ptr(), wsb, s, fa.data_ptr())
        assert (lib.msl_bn_fwd_mask(*fargs, bits.data_ptr()) if use_bits else lib.msl_bn_fwd_am(*fargs)) == 0
        dx, dres = torch.empty_like(x), torch.empty_like(x)
        dg, db = torch.empty(c, device=DEV), torch.empty(c, device=DEV)
        tail = (gamma.data_ptr(), beta.data_ptr(), sm.data_ptr(), si.data_ptr(), dx.data_ptr(), dres.data_ptr(),
                dg.data_ptr(), db.data_ptr(), c, p, nimg, 1, 1, 0, hip.forms(), ws.data_ptr(), wsb, s, ba.data_ptr())
        if use_bits:
            assert lib.msl_bn_bwd_mask(gy.data_ptr(), x.data_ptr(), bits.data_ptr(), *tail) == 0
        else:
            assert lib.msl_bn_bwd_am_beta(gy.data_ptr(), x.data_ptr(), y.data_ptr(), *tail) == 0
        torch.cuda.synchronize()
        outs.append((y, sm, si, rm, rv, fa, dx, dres, dg, db, ba))
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    y = outs[1][0]
    assert 0.2 < (y == 0).float().mean().item() < 0.8  # the mask matters
    pos = (y > 0).reshape(c * nimg, p).cpu().numpy()
    pos = np.pad(pos, ((0, 0), (0, nw * 64 - p)))
    want = np.packbits(pos, axis=-1, bitorder="little").view("<u8").reshape(-1)
    assert np.array_equal(bits.cpu().numpy().view("<u8"), want)
    # refusals: bits need relu and the fused kernels
    args_norelu = list(fargs[:17]) + [0] + list(fargs[18:])
    assert lib.msl_bn_fwd_mask(*args_norelu, bits.data_ptr()) == -3
    prev = ops.set_bn_fused(False)
    try:
        assert lib.msl_bn_fwd_mask(*fargs, bits.data_ptr()) == -3
        assert lib.msl_bn_bwd_mask(gy.data_ptr(), x.data_ptr(), bits.data_ptr(), *tail) == -3
    finally:
        ops.set_bn_fused(prev)


# ---------------------------------------------------------------------------- stem / maxpool / stride 2
@pytest.mark.parametrize("h,w", [(64, 128), (33, 47), (512, 1024)])
def test_stem_conv_fwd_bwd(h, w, f32_form):
    """ResNetMulti.conv1 (7x7, stride 2, pad 3) as im2col + the pointwise GEMM: output, data and weight
    gradients against fp64 (deeplab_multi.py:73-74)."""
    g = torch.Generator().manual_seed(h + w)
    x = torch.randn(1, 3, h, w, generator=g) * 50
    wt = torch.randn(64, 3, 7, 7, generator=g) * 0.01
    ho, wo = (h - 1) // 2 + 1, (w - 1) // 2 + 1
    gy = torch.randn(1, 64, ho, wo, generator=g)
    xr, wr = x.double().requires_grad_(), wt.double().requires_grad_()
    yr = F.conv2d(xr, wr, stride=2, padding=3)
    yr.backward(gy.double())
    xg, wg = x.to(DEV).requires_grad_(), wt.to(DEV).requires_grad_()
    y = ops.stem_conv(xg, wg, 2, 3, ops.PackCache(pointwise=True))
    assert y.shape == yr.shape
    y.backward(gy.to(DEV))
    torch.cuda.synchronize()
    assert _rel(y, yr) < 1e-5
    assert _rel(xg.grad, xr.grad) < 1e-5
    assert _rel(wg.grad, wr.grad) < 1e-5


@pytest.mark.parametrize("h,w,nimg", [(64, 128, 1), (33, 47, 2), (512, 1024, 2)])
def test_stem_image_partials_same_bits(h, w, nimg):
    """r05: the stem GEMM takes its f16x3 operand scale from the image's absmax partials (max |col| =
    max |x|: every pixel lies in a window) - the same output bits as the column matrix's own partials."""
    from maxsquareloss_amd import hip
    lib = hip.load()
    prev = ops.set_f32_form("f16x3")
    try:
        g = torch.Generator().manual_seed(h * w + nimg)
        x = (torch.randn(1, 3, nimg, h, w, generator=g) * 50).to(DEV)
        wt = (torch.randn(64, 3, 7, 7, generator=g) * 0.01).to(DEV)
        cache = ops.PackCache(pointwise=True)
        y = ops.stem_conv(x, wt, 2, 3, cache)
        ho, wo = (h - 1) // 2 + 1, (w - 1) // 2 + 1
        p = ho * wo * nimg
        s = hip.stream_ptr()
        col = torch.empty(1, 147, nimg, ho, wo, device=DEV)
        assert lib.msl_im2col(x.data_ptr(), 3, h, w, nimg, 7, 7, 2, 3, 1, ho, wo, col.data_ptr(), s) == 0
        part = torch.empty(147, device=DEV)
        assert lib.msl_absmax_partials(col.data_ptr(), 147, p, part.data_ptr(), s) == 0
        yc = torch.empty_like(y)
        wsb = lib.msl_pconv_fwd_workspace(147, 64, p)
        ws = hip.workspace(wsb, DEV)
        packed = cache.get([wt.contiguous()], 147, 64, 0)
        assert lib.msl_pconv_fwd_sc(col.data_ptr(), packed.data_ptr(), yc.data_ptr(), 147, 64, p, hip.forms(),
                                    ws.data_ptr(), wsb, s, part.data_ptr(), 147) == 0
        torch.cuda.synchronize()
        assert torch.equal(part.max(), x.abs().max())
        assert torch.equal(y, yc)
    finally:
        ops.set_f32_form(prev)


@pytest.mark.parametrize("c,h,w,ceil", [(64, 256, 512, True), (5, 17, 33, True), (3, 16, 16, True),
                                        (4, 15, 20, False), (2, 7, 9, True)])
def test_maxpool_bit_exact(c, h, w, ceil):
    """MaxPool2d(3, 2, 1, ceil_mode) (deeplab_multi.py:77): output, argmax and gradient bit-exact
    against torch-CPU, with ties (quantised values), NaNs and -inf in the input."""
    g = torch.Generator().manual_seed(c * h + w)
    x = torch.relu(torch.randint(-3, 5, (1, c, h, w), generator=g).float())  # many exact ties
    x.view(-1)[::97] = float("nan")
    x.view(-1)[5::89] = float("-inf")
    gy = None
    xr = x.clone().requires_grad_()
    yr = F.max_pool2d(xr, 3, 2, 1, ceil_mode=ceil)
    gy = torch.randn(yr.shape, generator=g)
    yr.backward(gy)
    xg = x.to(DEV).requires_grad_()
    y = ops.maxpool2d(xg, 3, 2, 1, ceil)
    y.backward(gy.to(DEV))
    torch.cuda.synchronize()
    assert y.shape == yr.shape
    assert torch.equal(y.cpu().nan_to_num(7.0), yr.detach().nan_to_num(7.0))
    assert torch.equal(xg.grad.cpu(), xr.grad)


def test_subsample_and_strided_pointwise(f32_form):
    """x[:, :, ::2, ::2] and the stride-2 1x1 convs of layer2.0 (deeplab_multi.py:12-13, 96-99):
    forward and gradients against fp64 F.conv2d(stride=2)."""
    from maxsquareloss_amd.graphs.models import deeplab_multi as dm
    g = torch.Generator().manual_seed(9)
    x = torch.randn(1, 256, 33, 65, generator=g)
    conv = dm.PointwiseConv(256, 512, stride=2).to(DEV)
    wt = conv.weight.detach().cpu()
    xr, wr = x.double().requires_grad_(), wt.double().requires_grad_()
    yr = F.conv2d(xr, wr, stride=2)
    gy = torch.randn(yr.shape, generator=g)
    yr.backward(gy.double())
    xg = x.to(DEV).requires_grad_()
    y = conv(xg)
    y.backward(gy.to(DEV))
    torch.cuda.synchronize()
    assert y.shape == yr.shape
    assert _rel(y, yr) < 1e-5 and _rel(xg.grad, xr.grad) < 1e-5 and _rel(conv.weight.grad, wr.grad) < 1e-5
    s = ops.subsample(x.to(DEV), 2)
    assert torch.equal(s.cpu(), x[:, :, ::2, ::2])
