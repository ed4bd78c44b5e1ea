"""ORACLE - test infrastructure only (tests/, __graft_entry__.smoke(), bench.py cpu_baseline).

A CPU restatement of the reference's hot path in plain PyTorch-CPU ops, written
from the reference's behaviour (cited file:line, paths relative to the
reference root) - it shares no code with the HIP product path and nothing in
maxsquareloss_amd/ may import it.

  forward()            graphs/models/deeplab_multi.py:8-130 (Bottleneck, ASPP with the
                       early return of :63-66 (Q1), bilinear align_corners upsample)
  ce()                 nn.CrossEntropyLoss(ignore_index=-1), train_source.py:128
  maxsquare()          utils/loss.py:104-119
  iw_maxsquare()       utils/loss.py:69-102 (histc on the host, :92-96)
  multi_guidance_ce()  tools/solve_gta5.py:206-213
  SGDMult              torch.optim.SGD single-tensor loop over optim_parameters()
                       (train_source.py:139-144; deeplab_multi.py:132-171; quirk Q2)
  uda_step()           tools/solve_gta5.py:335-387
  source_step()        tools/train_source.py:233-264
  image_transform()    datasets/cityscapes_Dataset.py:14, 245-251 (numpy_transform)
  label_transform()    datasets/cityscapes_Dataset.py:141-155, 260-264 (id2trainId)

Pinned against the real reference: tests/golden/*.npz are produced by
oracle/gen_golden.py, which imports the reference's own deeplab_multi.py and
loss.py by path in the survey container (and its SGD semantics through
torch.optim.SGD(foreach=False)); tests/test_oracle_golden.py checks this module
against them.
"""
import numpy as np
import torch
import torch.nn.functional as F

LAYERS = [3, 4, 23, 3]
PLANES = [64, 128, 256, 512]
STRIDES = [1, 2, 1, 1]
DILATIONS = [1, 1, 2, 4]
ASPP_DIL = [6, 12, 18, 24]


# --------------------------------------------------------------------------- parameters
def param_specs(num_classes):
    """[(name, shape, kind)] in the reference's registration order (named_parameters())."""
    specs = [("conv1.weight", (64, 3, 7, 7), "conv"), ("bn1.weight", (64,), "bnw"), ("bn1.bias", (64,), "bnb")]
    inplanes = 64
    for li, (planes, n, stride, dil) in enumerate(zip(PLANES, LAYERS, STRIDES, DILATIONS)):
        for b in range(n):
            pre = f"layer{li + 1}.{b}."
            cin = inplanes if b == 0 else planes * 4
            specs += [(pre + "conv1.weight", (planes, cin, 1, 1), "conv"), (pre + "bn1.weight", (planes,), "bnw"),
                      (pre + "bn1.bias", (planes,), "bnb"), (pre + "conv2.weight", (planes, planes, 3, 3), "conv"),
                      (pre + "bn2.weight", (planes,), "bnw"), (pre + "bn2.bias", (planes,), "bnb"),
                      (pre + "conv3.weight", (planes * 4, planes, 1, 1), "conv"),
                      (pre + "bn3.weight", (planes * 4,), "bnw"), (pre + "bn3.bias", (planes * 4,), "bnb")]
            if b == 0:
                specs += [(pre + "downsample.0.weight", (planes * 4, cin, 1, 1), "conv"),
                          (pre + "downsample.1.weight", (planes * 4,), "bnw"),
                          (pre + "downsample.1.bias", (planes * 4,), "bnb")]
        inplanes = planes * 4
    for head, cin in (("layer5", 1024), ("layer6", 2048)):
        for i in range(4):
            specs += [(f"{head}.conv2d_list.{i}.weight", (num_classes, cin, 3, 3), "conv"),
                      (f"{head}.conv2d_list.{i}.bias", (num_classes,), "aspp_bias")]
    return specs


def bn_names(num_classes):
    return [n[:-len(".weight")] for n, _, k in param_specs(num_classes) if k == "bnw"]


def multiplicity(name):
    """Occurrences of a parameter in optim_parameters() (deeplab_multi.py:139-171, Q2).
    Returns (group, k); bn1 (requires_grad=False, :76-77) -> (0, 0)."""
    if name.startswith("bn1."):
        return 0, 0
    if name == "conv1.weight":
        return 0, 1
    if name.startswith("layer5.") or name.startswith("layer6."):
        return 1, 1
    return 0, 4 if ".downsample." in name else 3


def optim_param_lists(names):
    """The two group lists with duplicates, in the reference's generator order."""
    g0 = []
    order = ["conv1", "bn1", "layer1", "layer2", "layer3", "layer4"]
    by_prefix = {p: [n for n in names if n.split(".")[0] == p] for p in order}
    # b[i].modules() walks the module tree depth-first, each module yielding ALL its (recursive) params
    for top in order:
        pn = by_prefix[top]
        if top in ("conv1", "bn1"):
            g0 += [n for n in pn if multiplicity(n)[1] > 0]
            continue
        g0 += pn  # the Sequential itself
        blocks = sorted({int(n.split(".")[1]) for n in pn})
        for b in blocks:
            bp = [n for n in pn if n.split(".")[1] == str(b)]
            g0 += bp  # the Bottleneck
            subs = []
            for n in bp:
                sub = n.split(".")[2]
                if sub not in subs:
                    subs.append(sub)
            for sub in subs:
                sp = [n for n in bp if n.split(".")[2] == sub]
                if sub == "downsample":
                    g0 += sp  # the downsample Sequential
                    for leaf in ("0", "1"):
                        g0 += [n for n in sp if n.split(".")[3] == leaf]
                else:
                    g0 += sp
    g1 = [n for n in names if n.startswith("layer5.") or n.startswith("layer6.")]
    return g0, g1


# --------------------------------------------------------------------------- fp16-operand convs
def round_f16(t, dim=None):
    """t rounded to fp16 as the fp16 MFMA path rounds its operands: scaled by a power of two that
    puts the absolute maximum (of the tensor, or of each slice along `dim`) into [2^14, 2^15),
    rounded to nearest-even fp16, unscaled - every step exact except the rounding itself."""
    a = t.detach().abs()
    if dim is None:
        m = a.max()
    else:
        m = a.transpose(0, dim).reshape(t.shape[dim], -1).max(1)[0]
        m = m.view([-1 if i == dim else 1 for i in range(t.dim())])
    m = torch.where(m > 0, m, torch.ones_like(m))
    sc = torch.ldexp(torch.ones_like(m), 15 - torch.frexp(m).exponent)
    return ((t * sc).half().to(t.dtype)) / sc


class _ConvF16(torch.autograd.Function):
    """F.conv2d with the operands of every product rounded to fp16 (round_f16), products summed in
    the working precision: the emulation of BASELINE config 5's fp16 MFMA convs.
      forward        x (one scale per tensor) * W (one scale per tensor)
      data gradient  dy (per tensor) * W
      weight grad    dy (one scale per output channel) * x (one per input channel) when
                     `wgrad_rounds(cin, cout, h, w)` says so, else exact - as the kernels choose."""

    @staticmethod
    def forward(ctx, x, w, b, stride, padding, dilation, wgrad_rounds):
        ctx.save_for_backward(x, w)
        ctx.conf = (stride, padding, dilation, b is not None, wgrad_rounds)
        return F.conv2d(round_f16(x), round_f16(w), b, stride, padding, dilation)

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        stride, padding, dilation, has_b, wgrad_rounds = ctx.conf
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            gx = torch.nn.grad.conv2d_input(x.shape, round_f16(w), round_f16(gy), stride, padding, dilation)
        if ctx.needs_input_grad[1]:
            rnd = wgrad_rounds(w.shape[1], w.shape[0], w.shape[2], gy.shape[2], gy.shape[3])
            xr, gr = (round_f16(x, 1), round_f16(gy, 1)) if rnd else (x, gy)
            gw = torch.nn.grad.conv2d_weight(xr, w.shape, gr, stride, padding, dilation)
        if has_b and ctx.needs_input_grad[2]:
            gb = gy.sum((0, 2, 3))
        return gx, gw, gb, None, None, None, None


def conv_f16(wgrad_rounds):
    """A conv2d(x, w, b, stride, padding, dilation) in the fp16-operand emulation (_ConvF16)."""
    def conv(x, w, b=None, stride=1, padding=0, dilation=1):
        return _ConvF16.apply(x, w, b, stride, padding, dilation, wgrad_rounds)
    return conv


def _split_gemm_rounds(m, n, ntap, p, row):
    """Whether a weight-gradient GEMM dW[m][n][tap] = sum_p dY[m][p] X[n][p + shift] of the fp16 path runs on
    the split kernel (both operands rounded to fp16, one power-of-two scale per row) rather than the exact
    bf16x6 one.  The rule DESIGN.md §3.3 states for k_wgrad_x6: 128 x 128 tiles, so at least 128 rows on
    both sides; 16-pixel K-steps whose image-border masks handle one row wrap, so image rows of at least 16
    pixels (a pointwise call passes the whole pixel axis as one row); and either at least 256 channels on
    both sides or chunked split-K items - (tile, pixel chunk) pairs of >= 8 K-steps, <= 4096 items - that
    fill at least 75 % of the 512 resident workgroups in their last round."""
    if m < 128 or n < 128 or row < 16:
        return False
    ntiles = -(-m // 128) * -(-n // 128) * ntap
    ks = -(-p // 16)
    best = 0.0
    for c in range(1, ks + 1):
        if ntiles * c > 4096:
            break
        length = -(-ks // c)
        if length < 8:
            break
        items = ntiles * -(-ks // length)
        fill = items / (-(-items // 512) * 512)
        if fill > best + 0.01:
            best = fill
    return best >= 0.75 or (m >= 256 and n >= 256)


def f16_wgrad_rounds(num_classes, nimg=2, aspp_shift=True):
    """The fp16 emulation's weight-gradient predicate (cin, cout, k, h, w) -> bool for _ConvF16 at the
    trainer's shapes (image pairs: nimg = 2; h x w = the gradient's map), restated from the design rule
    (_split_gemm_rounds) instead of asked of the library (r06; tests/test_host.py holds it
    equal to msl_conv_wgrad_split on every conv of the three config sizes):
      - 3x3: M = cout, N = cin, 9 taps, rows of w pixels;
      - 1x1: one flat row of nimg * h * w pixels; with more output than input channels the GEMM runs on
        swapped operands (the narrower one pre-split), so M = cin, N = cout there - the rule then asks the
        swapped shape first;
      - the ASPP heads in the shift form: one pointwise GEMM of 18 * classes rows over the 2048 / 1024-channel
        map (the 3x3 weight gradient is scattered from it)."""
    def rounds(cin, cout, k, h, w):
        p = nimg * h * w
        if k == 3 and cout == num_classes and aspp_shift:
            cout, k = 18 * num_classes, 1
        if k == 1:
            if cout > cin and _split_gemm_rounds(cin, cout, 1, p, p):
                return True
            return _split_gemm_rounds(cout, cin, 1, p, p)
        return _split_gemm_rounds(cout, cin, 9, p, w)
    return rounds


def conv_calls(H, W, num_classes):
    """(cin, cout, k, h_out, w_out) of every conv that forward_low runs through its `conv` argument (the stem
    stays fp32 and is not one of them) for an H x W image, in call order - taken from the model's own forward
    on the meta device, so the geometry (stride-2 1x1s, ceil-mode pooling) is the model's."""
    calls = []

    def rec(x, w, b=None, stride=1, padding=0, dilation=1):
        y = F.conv2d(x, w, b, stride, padding, dilation)
        calls.append((w.shape[1], w.shape[0], w.shape[2], y.shape[2], y.shape[3]))
        return y
    meta = torch.device("meta")
    params = {n: torch.empty(s, device=meta) for n, s, _ in param_specs(num_classes)}
    buffers = {}
    for n in bn_names(num_classes):
        c = params[n + ".weight"].shape[0]
        buffers[n + ".running_mean"] = torch.zeros(c, device=meta)
        buffers[n + ".running_var"] = torch.ones(c, device=meta)
    forward_low(params, buffers, torch.empty(1, 3, H, W, device=meta), True, rec)
    return calls


# --------------------------------------------------------------------------- forward
def _bn(x, params, buffers, name, training):
    return F.batch_norm(x, buffers[name + ".running_mean"], buffers[name + ".running_var"],
                        params[name + ".weight"], params[name + ".bias"], training, 0.1, 1e-5)


def _bottleneck(x, params, buffers, pre, stride, dil, has_down, training, conv=F.conv2d):
    out = conv(x, params[pre + "conv1.weight"], stride=stride)
    out = F.relu(_bn(out, params, buffers, pre + "bn1", training))
    out = conv(out, params[pre + "conv2.weight"], padding=dil, dilation=dil)
    out = F.relu(_bn(out, params, buffers, pre + "bn2", training))
    out = conv(out, params[pre + "conv3.weight"])
    out = _bn(out, params, buffers, pre + "bn3", training)
    res = x
    if has_down:
        res = conv(x, params[pre + "downsample.0.weight"], stride=stride)
        res = _bn(res, params, buffers, pre + "downsample.1", training)
    return F.relu(out + res)


def _aspp(x, params, head, conv=F.conv2d):
    # Classifier_Module.forward returns after the first loop iteration (deeplab_multi.py:63-66)
    out = conv(x, params[f"{head}.conv2d_list.0.weight"], params[f"{head}.conv2d_list.0.bias"],
               padding=ASPP_DIL[0], dilation=ASPP_DIL[0])
    return out + conv(x, params[f"{head}.conv2d_list.1.weight"], params[f"{head}.conv2d_list.1.bias"],
                      padding=ASPP_DIL[1], dilation=ASPP_DIL[1])


def features(params, buffers, x, training=True):
    x = F.conv2d(x, params["conv1.weight"], stride=2, padding=3)
    x = F.relu(_bn(x, params, buffers, "bn1", training))
    x = F.max_pool2d(x, 3, 2, 1, ceil_mode=True)
    low = {}
    for li, (n, stride, dil) in enumerate(zip(LAYERS, STRIDES, DILATIONS)):
        for b in range(n):
            x = _bottleneck(x, params, buffers, f"layer{li + 1}.{b}.", stride if b == 0 else 1, dil, b == 0, training)
        low[li + 1] = x
    return low


def forward_low(params, buffers, x, training=True, conv=F.conv2d):
    """(x2_low, x1_low): the ASPP outputs before upsampling.  `conv` runs every conv but the stem
    (conv_f16: the fp16 path, whose stem stays fp32)."""
    x = F.conv2d(x, params["conv1.weight"], stride=2, padding=3)
    x = F.relu(_bn(x, params, buffers, "bn1", training))
    x = F.max_pool2d(x, 3, 2, 1, ceil_mode=True)
    for li in range(3):
        for b in range(LAYERS[li]):
            x = _bottleneck(x, params, buffers, f"layer{li + 1}.{b}.", STRIDES[li] if b == 0 else 1,
                            DILATIONS[li], b == 0, training, conv)
    x1 = _aspp(x, params, "layer5", conv)
    for b in range(LAYERS[3]):
        x = _bottleneck(x, params, buffers, f"layer4.{b}.", 1, DILATIONS[3], b == 0, training, conv)
    x2 = _aspp(x, params, "layer6", conv)
    return x2, x1


def forward(params, buffers, x, training=True, conv=F.conv2d):
    """ResNetMulti.forward (deeplab_multi.py:113-130) -> (x2, x1) upsampled to the input size."""
    hw = x.shape[2:]
    x2, x1 = forward_low(params, buffers, x, training, conv)
    up = lambda t: F.interpolate(t, size=hw, mode="bilinear", align_corners=True)  # noqa: E731
    return up(x2), up(x1)


# --------------------------------------------------------------------------- losses
def ce(pred, y):
    return F.cross_entropy(pred, y, ignore_index=-1)


def maxsquare(prob):
    mask = prob != -1  # always true (Q5)
    return -torch.mean(torch.pow(prob, 2)[mask]) / 2


def iw_hist_weights(prob, ratio, num_class, label=None):
    maxpred, argpred = torch.max(prob, 1)
    if label is None:
        label = argpred
    hist = torch.histc(label[0].detach().cpu().float(), bins=num_class + 1, min=-1, max=num_class - 1)[1:]
    w = 1 / torch.max(torch.pow(hist, ratio) * torch.pow(hist.sum(), 1 - ratio), torch.ones(1))
    return hist, w, argpred


def iw_maxsquare(prob, ratio, num_class, label=None):
    hist, w, argpred = iw_hist_weights(prob, ratio, num_class, label)
    weights = w[argpred[0]].detach().unsqueeze(0)
    n = prob.size(0)
    return -torch.sum(torch.pow(prob, 2) * weights) / (n * num_class), hist


def multi_guidance_label(P, P2, threshold):
    maxpred, _ = torch.max(P.detach(), dim=1)
    maxpred_2, _ = torch.max(P2.detach(), dim=1)
    pred_c = (P + P2) / 2
    _, argpred_c = torch.max(pred_c, dim=1)
    mask = (maxpred > threshold) | (maxpred_2 > threshold)
    return torch.where(mask, argpred_c, torch.full_like(argpred_c, -1))


def multi_guidance_ce(pred, pred_2, threshold):
    P = F.softmax(pred, dim=1)
    P2 = F.softmax(pred_2, dim=1)
    return ce(pred_2, multi_guidance_label(P, P2, threshold))


# --------------------------------------------------------------------------- SGD
class SGDMult:
    """torch.optim.SGD(momentum, weight_decay) single-tensor semantics over the duplicated
    group lists: k sequential updates, one shared buffer, fresh buffer per occurrence on the
    first step (the last kept).  Parameters whose grad is None are skipped."""

    def __init__(self, params, names, lr, momentum=0.9, weight_decay=5e-4):
        self.params = params
        g0, g1 = optim_param_lists(names)
        self.groups = [{"names": g0, "lr": lr}, {"names": g1, "lr": 10 * lr}]
        self.momentum, self.wd = momentum, weight_decay
        self.buf = {}

    @torch.no_grad()
    def step(self):
        for g in self.groups:
            lr = g["lr"]
            bufs = [self.buf.get(n) for n in g["names"]]
            for i, n in enumerate(g["names"]):
                p = self.params[n]
                if p.grad is None:
                    continue
                d = p.grad.add(p, alpha=self.wd)
                if self.momentum != 0:
                    b = bufs[i]
                    if b is None:
                        b = torch.clone(d).detach()
                        bufs[i] = b
                    else:
                        b.mul_(self.momentum).add_(d)
                    d = b
                p.add_(d, alpha=-lr)
            for n, b in zip(g["names"], bufs):
                if b is not None:
                    self.buf[n] = b

    def zero_grad(self):
        for p in self.params.values():
            p.grad = None


# --------------------------------------------------------------------------- steps
class Model:
    """Parameters + BN buffers as plain tensors (state_dict naming of DeeplabMulti)."""

    def __init__(self, state_dict, num_classes=19, dtype=torch.float32, f16_wgrad=None):
        """f16_wgrad: None = the reference's arithmetic; a predicate (cin, cout, k, h, w) -> bool =
        the fp16-operand emulation of config 5's conv path (conv_f16), the predicate telling which
        weight gradients round their operands."""
        self.num_classes = num_classes
        self.dtype = dtype
        self.conv = F.conv2d if f16_wgrad is None else conv_f16(f16_wgrad)
        names = [n for n, _, _ in param_specs(num_classes)]
        self.names = names
        self.params = {n: state_dict[n].detach().clone().to(dtype) for n in names}
        for n in names:
            self.params[n].requires_grad_(multiplicity(n)[1] > 0)
        self.buffers = {k: (v.detach().clone().to(dtype) if v.is_floating_point() else v.detach().clone())
                        for k, v in state_dict.items() if k not in self.params}

    def __call__(self, x, training=True):
        return forward(self.params, self.buffers, x.to(self.dtype), training, self.conv)

    def state_dict(self):
        sd = {n: p.detach() for n, p in self.params.items()}
        sd.update(self.buffers)
        return sd


def poly_lr(init_lr, it, max_iter, power=0.9):
    """train_source.py:706-717."""
    return init_lr * (1 - float(it) / max_iter) ** power


def uda_step(model, opt, xs, ys, xt, cfg, it):
    """One iteration of solve_gta5.py:335-387.  cfg keys: lr, iter_max, target_mode
    ('maxsquare'|'IW_maxsquare'), multi, lambda_seg, lambda_target, IW_ratio, threshold."""
    lr = poly_lr(cfg["lr"], it, cfg["iter_max"])
    opt.groups[0]["lr"], opt.groups[1]["lr"] = lr, 10 * lr
    out = uda_grads(model, xs, ys, xt, cfg)
    opt.step()
    opt.zero_grad()
    return out


def uda_grads(model, xs, ys, xt, cfg):
    """The two forward/backward passes of uda_step (solve_gta5.py:344-381) without the optimizer step:
    the gradients accumulate into the parameters' .grad (a data-parallel replica's local part)."""
    out = {}
    pred, pred_2 = model(xs)
    loss_s = ce(pred, ys)
    loss_ = loss_s
    if cfg["multi"]:
        loss_2 = cfg["lambda_seg"] * ce(pred_2, ys)
        loss_ = loss_ + loss_2
        out["loss_seg_2"] = loss_2.item()
    loss_.backward()
    out["loss_seg"] = loss_s.item()
    pred, pred_2 = model(xt)
    P = F.softmax(pred, dim=1)
    if cfg["target_mode"] == "maxsquare":
        lt = maxsquare(P)
    elif cfg["target_mode"] == "IW_maxsquare":
        lt, hist = iw_maxsquare(P, cfg["IW_ratio"], model.num_classes)
        out["hist"] = hist.numpy().astype(np.int64)
    else:
        raise ValueError(cfg["target_mode"])
    loss_t = cfg["lambda_target"] * lt
    total = loss_t
    if cfg["multi"]:
        lt2 = cfg["lambda_seg"] * cfg["lambda_target"] * multi_guidance_ce(pred, pred_2, cfg["threshold"])
        total = total + lt2
        out["loss_target_2"] = lt2.item()
    total.backward()
    out["loss_target"] = loss_t.item()
    return out


def source_step(model, opt, x, y, cfg, it):
    """train_source.py:233-264 (one iteration of the source-only trainer)."""
    lr = poly_lr(cfg["lr"], it, cfg["iter_max"])
    opt.groups[0]["lr"], opt.groups[1]["lr"] = lr, 10 * lr
    pred, pred_2 = model(x)
    cur = ce(pred, y)
    if cfg["multi"]:
        cur = cur + cfg["lambda_seg"] * ce(pred_2, y)
    opt.zero_grad()
    cur.backward()
    opt.step()
    return {"loss": cur.item()}


# ----------------------------------------------------------------------------- evaluation
# utils/eval.py:109-115 (__generate_matrix) and :25-98 (the metrics), restated in numpy.
def confusion(gt, pred_logits, num_class):
    """np.argmax over classes of pred [C, H, W], then bincount of num_class*gt + argmax over the
    pixels with 0 <= gt < num_class (utils/eval.py:111-114; train_source.py:280-282)."""
    arg = np.argmax(pred_logits.reshape(num_class, -1), axis=0)
    g = gt.reshape(-1)
    keep = (g >= 0) & (g < num_class)
    idx = num_class * g[keep].astype(np.int64) + arg[keep]
    return np.bincount(idx, minlength=num_class ** 2).reshape(num_class, num_class), arg


_S16 = [0, 1, 2, 3, 4, 5, 6, 7, 8, 10, 11, 12, 13, 15, 17, 18]   # utils/eval.py:9
_S13 = [0, 1, 2, 6, 7, 8, 10, 11, 12, 13, 15, 17, 18]             # :10
_S16_13 = [0, 1, 2, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15]           # :11


def eval_metrics(cm, out_16_13=False):
    """PA, MPA, MIoU, FWIoU, Precision of utils/eval.py:25-98 for a [C, C] float matrix (the
    16-class SYNTHIA case returns (16, 13) pairs as the reference does)."""
    cm = np.asarray(cm, dtype=np.float64)
    n = cm.shape[0]
    with np.errstate(divide="ignore", invalid="ignore"):
        diag, rows, cols = np.diag(cm), cm.sum(axis=1), cm.sum(axis=0)
        pa = 0 if cm.sum() == 0 else diag.sum() / cm.sum()
        mpa, iou, prec = diag / rows, diag / (rows + cols - diag), diag / cols
        fw = rows * iou

    def mean(v):
        if n == 16:
            return np.nanmean(v), np.nanmean(v[_S16_13])
        if out_16_13:
            return np.nanmean(v[_S16]), np.nanmean(v[_S13])
        return np.nanmean(v)

    def fwsum(v):
        tot = cm.sum()
        if n == 16:
            return sum(x for x in v if not np.isnan(x)) / tot, sum(x for x in v[_S16_13] if not np.isnan(x)) / tot
        if out_16_13:
            return sum(x for x in v[_S16] if not np.isnan(x)) / tot, sum(x for x in v[_S13] if not np.isnan(x)) / tot
        return sum(x for x in v if not np.isnan(x)) / tot

    return {"PA": pa, "MPA": mean(mpa), "MIoU": mean(iou), "FWIoU": fwsum(fw), "Precision": mean(prec)}


# ----------------------------------------------------------------------------- input pipeline
def image_transform(rgb, mean, mirror=False):
    """cityscapes_Dataset.py:245-251 with numpy_transform: uint8 RGB HWC -> float32, BGR,
    minus IMG_MEAN (float32), CHW; mirror = Image.FLIP_LEFT_RIGHT first (:182)."""
    img = np.asarray(rgb[:, ::-1] if mirror else rgb, np.float32)
    img = img[:, :, ::-1] - np.asarray(mean, np.float32)
    return img.transpose(2, 0, 1).copy()


def label_transform(ids, id_to_trainid, set_16=None, set_13=None, mirror=False):
    """cityscapes_Dataset.py:141-155: ids -> trainIds (-1 for unlisted ids), then the optional
    16- or 13-class remap (trainIds outside the set -> -1)."""
    lab = np.asarray(ids[:, ::-1] if mirror else ids, np.float32)
    out = np.full(lab.shape, -1, np.float32)
    for k, v in id_to_trainid.items():
        out[lab == k] = v
    for sub in (set_16, set_13):
        if sub is not None:
            o2 = np.full(lab.shape, -1, np.float32)
            for i, t in enumerate(sub):
                o2[out == t] = i
            out = o2
    return out
