"""torch.autograd wrappers over the HIP kernels of libmsl_hip.so.

Each Function is a thin shim: shape checks on the host, then one or two C-ABI
calls on torch's current HIP stream.  Tensors are bs=1 NCHW fp32 (the
reference only runs bs=1: IW_MaxSquareloss broadcasts (N,H,W) weights against
(N,C,H,W) probabilities, which only works for N=1 - SURVEY.md quirk Q3), or an
image PAIR (1, C, 2, H, W): the source and target images of one UDA iteration laid
out [C][2][H][W], each image convolved, pooled and batch-normalised on its own (its
own bs=1 statistics) while every conv GEMM runs once over both (pair_join /
pair_split; the trunk ops take either form, the losses one image).
"""
import ctypes
from contextlib import nullcontext as _nullctx

import torch
from torch.autograd import Function

from . import hip

_f32 = torch.float32

# Conv MFMA precision: "fp32" (fp32-accurate, in the library's fp32 form below), "fp16"
# (v_mfma_f32_32x32x16_f16 on operands scaled by a power of two and rounded to fp16, fp32 sums:
# BASELINE config 5's fp16 MFMA path; needs the f16x3 fp32 form's packs) or "bf16"
# (v_mfma_f32_32x32x16_bf16 on operands rounded to bf16, fp32 sums).  Activations, BN, losses
# and the optimizer stay fp32 in every case.
CONV_MATH = "fp32"


def set_conv_math(math):
    global CONV_MATH
    if math not in ("fp32", "fp16", "bf16"):
        raise ValueError(f"conv math must be 'fp32', 'fp16' or 'bf16', got {math!r}")
    CONV_MATH = math


# Matrix-core form of the fp32 conv math (hip.FORMS.f32_form, passed with every conv / pack call as
# msl_forms): "mfma_f32" = v_mfma_f32_32x32x2_f32, an exact fmaf chain; "bf16x6" =
# each operand split into three bf16 terms, six products per 16-deep K slice on
# v_mfma_f32_32x32x16_bf16 with fp32 sums (fp32-accurate; csrc/dconv_kernels.h Split3); "f16x3" =
# each operand tensor scaled by a power of two and split into two fp16 terms, three products per
# slice on v_mfma_f32_32x32x16_f16 with fp32 sums (fp32-accurate; dconv_kernels.h Split2h).
F32_FORMS = {"mfma_f32": 0, "bf16x6": 2, "f16x3": 5}
SPLIT_FORMS = ("bf16x6", "f16x3")  # the forms the HIP pointwise / 128-row kernels run split


def _form_code():
    """The f32 form code the conv / pack calls pass (packs are form-specific: it keys the pack caches)."""
    return hip.FORMS.f32_form


def set_f32_form(form):
    """Select the fp32 conv form; returns the previous one."""
    if form not in F32_FORMS:
        raise ValueError(f"fp32 conv form must be one of {sorted(F32_FORMS)}, got {form!r}")
    prev = hip.set_form("f32_form", F32_FORMS[form])
    return {v: k for k, v in F32_FORMS.items()}[prev]


def set_bn_fused(fused):
    """Select the BN kernel form (msl_forms.bn_fused): True = one fused launch per train-mode BN
    call on maps of <= 16384 px (<= 33792 px with >= 128 channels); returns the previous setting."""
    return bool(hip.set_form("bn_fused", int(bool(fused))))


def f32_form():
    return {v: k for k, v in F32_FORMS.items()}[hip.FORMS.f32_form]


def _fn(lib, name, math):
    return getattr(lib, name + "_bf16") if math == "bf16" else getattr(lib, name)


def _h3(math="fp32"):
    """Whether the conv GEMMs of this math scale their operands (and so read absmax partials)."""
    return math == "fp16" or (math == "fp32" and _form_code() == F32_FORMS["f16x3"])


def _tag_absmax(t, part):
    """Attach the per-channel absmax partials a BN kernel wrote for its output `t` (msl_bn_*_am)."""
    t._msl_absmax = (part, t._version)


def _parts(t, math="fp32", compute=True):
    """The per-channel absmax partials of an operand tensor for the f16x3 form, as (tensor, count =
    channels): the ones the BN kernel that produced `t` wrote (msl_bn_fwd_am / msl_bn_bwd_am, no
    pass of their own), else - when `compute` - msl_absmax_partials, so that a tensor two GEMMs read
    (x: forward and weight gradient; dy: data and weight gradient) is reduced once.  None in the other
    forms (the kernels ignore them), or when not worth a launch (the entry point then reduces the
    operand itself if its kernel needs it)."""
    if not _h3(math):
        return None
    rec = getattr(t, "_msl_absmax", None)
    if rec is not None and rec[1] == t._version:
        return rec[0], rec[0].numel()
    if not compute:
        return None
    lib = hip.load()
    rows = t.size(1)
    part = torch.empty(rows, dtype=_f32, device=t.device)
    hip.check(lib.msl_absmax_partials(t.data_ptr(), rows, t.numel() // rows, part.data_ptr(), hip.stream_ptr()),
              "msl_absmax_partials")
    return part, rows


def _pp(q):
    """(pointer, count) of _parts' result for the _sc entry points."""
    return (None, 0) if q is None else (q[0].data_ptr(), q[1])


def _conv_call(lib, name, math, args, parts):
    """fp32: the _sc entry point, given the operands' absmax partials (None = the call reduces them
    itself; ignored outside f16x3); bf16: the _bf16 entry point."""
    if math == "bf16":
        return getattr(lib, name + "_bf16")(*args)
    suffix = "_f16" if math == "fp16" else "_sc"
    return getattr(lib, name + suffix)(*args, *(v for q in parts for v in _pp(q)))


def _split_gemm(m, k_other):
    """Whether a forward-form GEMM with M output rows runs a split (f16x3) kernel that scales its
    image operand (128-row tiles: M > 64), or a weight gradient of these channel counts the pre-split
    kernel (both >= 128): a partials launch only pays off where one of them reads the tensor."""
    return m > 64 or min(m, k_other) >= 128


def _check_act(x, name, images=False):
    """x contiguous; with `images`, (1,C,H,W) or an image batch (1,C,N,H,W) ([C][N][H][W])."""
    ok = x.is_cuda and x.dtype == _f32 and x.size(0) == 1 and (x.dim() == 4 or (images and x.dim() == 5))
    if not ok:
        shapes = "(1,C,H,W) or (1,C,N,H,W)" if images else "(1,C,H,W)"
        raise hip.MSLError(f"{name}: expected a CUDA fp32 tensor of shape {shapes}, got "
                           f"{tuple(x.shape)} {x.dtype} {x.device}")
    return x.contiguous()


def _nimg(x):
    """Images in an activation: 1 for (1,C,H,W), N for (1,C,N,H,W)."""
    return x.size(2) if x.dim() == 5 else 1


def _like(x, c, h, w, dtype=_f32):
    """An empty activation with x's image count and c channels of h x w."""
    shape = (1, c, x.size(2), h, w) if x.dim() == 5 else (1, c, h, w)
    return torch.empty(shape, dtype=dtype, device=x.device)


# --------------------------------------------------------------------------- gradient sinks
def grad_sink(p):
    """(grad view, FlatGrads, index) when `p`'s .grad is its slice of the optimizer's flat buffer.

    The backward of a HIP op then accumulates the weight gradient straight into that slice (the
    wgrad / BN kernels have an accumulate mode), notifies the flat buffer as AccumulateGrad's
    hook would (the data-parallel reducer listens there), and returns None for the parameter -
    saving autograd's separate `grad += new` kernel per parameter per backward.  Only for
    .backward()-driven training: torch.autograd.grad() on such a parameter would see None.
    """
    s = getattr(p, "_msl_flat", None)
    if s is None or p.grad is None or torch.is_grad_enabled():
        return None
    fg, i = s
    g = p.grad
    if g.data_ptr() != fg.flat.data_ptr() + 4 * int(fg.offsets[i]):
        return None
    return g, fg, i


# --------------------------------------------------------------------------- asynchronous weight gradients
# With ASYNC_WGRAD the weight gradients that accumulate in place into the flat gradient buffer (the
# training path: ops.grad_sink) run on a side stream per device, concurrently with the data-gradient
# chain of the backward (dgrad -> BN backward -> dgrad ...), which is latency-bound between its GEMMs.
# Everything that reads the flat buffer joins that stream first (wgrad_join: the SGD step, the data-
# parallel bucket launches, zero_grad).  Kernels, operands and per-buffer order are unchanged
# (results bit-identical).  Not in the reference, whose backward is one stream.  Off by default: the
# step measured slower with it (40.2 vs 39.5 ms same box: the concurrent GEMMs share the CUs and the
# caches; profiles/r03_async_wgrad_ab.txt).
ASYNC_WGRAD = False
_WG_STREAMS = {}


def _wgrad_stream(t):
    idx = t.device.index if t.device.index is not None else torch.cuda.current_device()
    ws = _WG_STREAMS.get(idx)
    if ws is None:
        ws = _WG_STREAMS[idx] = torch.cuda.Stream(device=t.device)
    ws.wait_stream(torch.cuda.current_stream(t.device))
    return ws


def _keep(ws, *tensors):
    """The side stream reads these: the caching allocator must not hand their memory to another
    stream's allocations before the side stream's work on them is done."""
    for t in tensors:
        if t is not None:
            t.record_stream(ws)


def wgrad_join(device=None):
    """Make the current stream wait for every weight gradient enqueued on the side stream."""
    if not _WG_STREAMS:
        return
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    ws = _WG_STREAMS.get(dev.index if dev.index is not None else torch.cuda.current_device())
    if ws is not None:
        torch.cuda.current_stream(dev).wait_stream(ws)


# --------------------------------------------------------------------------- packing cache
class PackCache:
    """Packed copies of a conv's weights, rebuilt when any weight changes.

    The forward GEMM wants W as [k = (tap, 16-channel block)][cout] and the
    data gradient wants the transposed, tap-flipped layout; both are derived
    from the parameters once per optimizer step (keyed on the tensors'
    in-place version counters), not once per call.
    """

    def __init__(self, pointwise=False):
        self.pointwise = pointwise
        self.key = {0: None, 1: None}
        self.buf = {0: None, 1: None}
        self.used = {0: False, 1: False}  # read by PackBatch: the directions a step consumes
        self.meta = {0: None, 1: None}    # (weights, cin, cout) of the last get()
        self._shift = None                # the ASPP shift form's packs (ops.aspp2)

    def shift_pack(self):
        if self._shift is None:
            self._shift = _ShiftPack()
        return self._shift

    @staticmethod
    def key_of(weights):
        return (_form_code(),) + tuple((w.data_ptr(), w._version) for w in weights)

    def get(self, weights, cin, cout, for_dgrad):
        key = self.key_of(weights)
        self.used[for_dgrad] = True
        self.meta[for_dgrad] = (list(weights), cin, cout)
        if self.key[for_dgrad] != key:
            lib = hip.load()
            nb = len(weights)
            if self.pointwise:
                total = lib.msl_pconv_packed_elems(cin, cout, for_dgrad)
            else:
                total = lib.msl_dconv_packed_elems(nb, cin, cout, for_dgrad)
            buf = self.buf[for_dgrad]
            if buf is None or buf.numel() != total or buf.device != weights[0].device:
                buf = torch.empty(total, dtype=_f32, device=weights[0].device)
            s = hip.stream_ptr()
            wc = [w.detach().contiguous() for w in weights]
            if self.pointwise:
                hip.check(lib.msl_pconv_pack(wc[0].data_ptr(), cin, cout, for_dgrad, buf.data_ptr(), hip.forms(), s),
                          "msl_pconv_pack")
            else:
                # one call packs every branch (and splits the bf16x6 planes behind them)
                stride = (wc[1].data_ptr() - wc[0].data_ptr()) // 4 if nb == 2 else 0
                if nb == 2 and (wc[1].data_ptr() - wc[0].data_ptr()) % 4:
                    raise hip.MSLError("dconv pack: misaligned branch weights")
                hip.check(lib.msl_dconv_pack(wc[0].data_ptr(), stride, nb, cin, cout, for_dgrad, buf.data_ptr(),
                                             hip.forms(), s),
                          "msl_dconv_pack")
            self.buf[for_dgrad] = buf
            self.key[for_dgrad] = key
        return self.buf[for_dgrad]


class PackBatch:
    """Every weight pack of a model in two launches (one per tap count) instead of one per conv
    and direction (~130 per training step): `run()` after the optimizer step packs each stale
    (PackCache, direction) that an earlier step consumed through msl_conv_pack_many
    (byte-identical to the per-conv calls) and marks it fresh.  The set of stale packs is the
    same every step (the parameters the loss reaches: with --multi False the layer3 ASPP head
    gets no gradient and keeps its packs), so the job tables are built once, outside graph
    capture (utils/graph.py captures iteration 1, after iteration 0 built them eagerly); a new
    set while capturing is left to PackCache.get's lazy path."""

    _JOB = None

    def __init__(self, module):
        self.caches = [m._pack for m in module.modules() if isinstance(getattr(m, "_pack", None), PackCache)]
        self.sig = None
        self.tables = {}
        self.launches = 0

    @classmethod
    def _dtype(cls):
        import numpy as np
        if cls._JOB is None:
            cls._JOB = np.dtype([("w", "<u8"), ("bs", "<i8"), ("packed", "<u8"), ("nb", "<i4"), ("cin", "<i4"),
                                 ("cout", "<i4"), ("fd", "<i4")])
            assert cls._JOB.itemsize == 40  # sizeof(msl_pack_job)
        return cls._JOB

    def _jobs(self):
        out = []
        for c in self.caches + [c._shift.pc for c in self.caches if c._shift is not None]:
            for d in (0, 1):
                if c.used[d] and c.buf[d] is not None and c.meta[d] is not None:
                    out.append((c, d))
        return out

    def _build(self, jobs, device):
        import numpy as np
        lib = hip.load()
        tables = {}
        for taps in (9, 1):
            sel = [(c, d) for c, d in jobs if (1 if c.pointwise else 9) == taps]
            if not sel:
                continue
            rec = np.zeros(len(sel), dtype=self._dtype())
            starts = np.zeros(len(sel) + 1, dtype=np.int64)
            for i, (c, d) in enumerate(sel):
                ws, cin, cout = c.meta[d]
                nb = len(ws)
                stride = 0
                if nb == 2:
                    diff = ws[1].data_ptr() - ws[0].data_ptr()
                    if diff % 4:
                        return None
                    stride = diff // 4
                if any(not w.is_contiguous() for w in ws):
                    return None
                rec[i] = (ws[0].data_ptr(), stride, c.buf[d].data_ptr(), nb, cin, cout, d)
                nblk = lib.msl_conv_pack_blocks(nb, taps, cin, cout, d)
                if nblk < 1:
                    return None
                starts[i + 1] = starts[i] + nblk
            jt = torch.from_numpy(rec.view(np.uint8).copy()).to(device)
            st = torch.from_numpy(starts).to(device)
            tables[taps] = (jt, st, len(sel), int(starts[-1]))
        return tables

    def run(self):
        for c in self.caches:  # the ASPP heads' shift-form layouts first (ops._ShiftPack): their packs follow
            if c._shift is not None and c._shift.meta is not None:
                c._shift.refresh()
        jobs, keys = [], []
        for c, d in self._jobs():
            k = c.key_of(c.meta[d][0])
            if c.key[d] != k:
                jobs.append((c, d))
                keys.append(k)
        if not jobs:
            return False
        sig = tuple((id(c), d, c.buf[d].data_ptr(), c.buf[d].numel(), tuple(w.data_ptr() for w in c.meta[d][0]),
                     c.meta[d][1], c.meta[d][2]) for c, d in jobs)
        if sig != self.sig:
            if torch.cuda.is_current_stream_capturing():
                return False
            tables = self._build(jobs, jobs[0][0].buf[jobs[0][1]].device)
            if tables is None:
                return False
            self.tables, self.sig = tables, sig
        lib = hip.load()
        s = hip.stream_ptr()
        for taps, (jt, st, n, total) in self.tables.items():
            hip.check(lib.msl_conv_pack_many(jt.data_ptr(), st.data_ptr(), n, taps, total, hip.forms(), s),
                      "msl_conv_pack_many")
        for (c, d), k in zip(jobs, keys):
            c.key[d] = k
        self.launches += 1
        return True


# --------------------------------------------------------------------------- dilated conv
# Live kernel timing for bench.py: PROBE[(nbranch, cin, cout, h, w, dil0)] = [] collects
# (start, end) HIP events recorded on the launching stream around each matching forward.
PROBE = {}


class _DConv3x3(Function):
    """sum_b conv3x3(x, W_b, dilation d_b) (+ sum_b bias_b); nbranch in {1, 2}."""

    @staticmethod
    def forward(ctx, x, w0, w1, b0, b1, dil0, dil1, cache):
        ctx.fm = hip.snapshot_forms()  # the backward runs the forms of its forward
        x = _check_act(x, "dconv3x3", images=True)
        n = _nimg(x)
        weights = [w0] if w1 is None else [w0, w1]
        nb = len(weights)
        cout, cin = w0.shape[0], w0.shape[1]
        if w0.shape[2:] != (3, 3) or x.size(1) != cin:
            raise hip.MSLError(f"dconv3x3: weight {tuple(w0.shape)} does not match input {tuple(x.shape)}")
        h, w = x.shape[-2], x.shape[-1]
        lib = hip.load()
        packed = cache.get(weights, cin, cout, 0)
        bias = None
        if b0 is not None:
            bias = torch.stack([b0] if nb == 1 else [b0, b1]).contiguous()
        y = _like(x, cout, h, w)
        wsb = lib.msl_dconv_fwd_workspace(nb, cin, cout, h, w, n)
        ws = hip.workspace(wsb, x.device)
        probe = PROBE.get((nb, cin, cout, h, w, dil0, n)) if PROBE else None
        if probe is not None:
            ev0 = torch.cuda.Event(enable_timing=True)
            ev0.record()
        math = CONV_MATH
        xpart = _parts(x, math, compute=_split_gemm(cout, cin))
        hip.check(_conv_call(lib, "msl_dconv_fwd", math,
                             (x.data_ptr(), packed.data_ptr(), hip.ptr(bias), y.data_ptr(), nb, cin, cout, h, w, n,
                              dil0, dil1 if nb > 1 else 0, hip.forms(), ws.data_ptr(), wsb,
                              hip.stream_ptr()), (xpart,)), "msl_dconv_fwd")
        if probe is not None:
            ev1 = torch.cuda.Event(enable_timing=True)
            ev1.record()
            probe.append((ev0, ev1))
        ctx.save_for_backward(x, *weights)
        ctx.meta = (nb, cin, cout, h, w, n, dil0, dil1, b0 is not None, cache, math)
        ctx.xpart = xpart
        return y

    @staticmethod
    def backward(ctx, gy):
        x, *weights = ctx.saved_tensors
        nb, cin, cout, h, w, n, dil0, dil1, has_bias, cache, math = ctx.meta
        gy = gy.contiguous()
        lib = hip.load()
        s = hip.stream_ptr()
        d1 = dil1 if nb > 1 else 0
        dx = None
        gpart = _parts(gy, math, compute=_split_gemm(cin, cout))
        xpart = ctx.xpart
        if ctx.needs_input_grad[0]:
            packed_d = cache.get(weights, cin, cout, 1)
            dx = torch.empty_like(x)
            wsb = lib.msl_dconv_dgrad_workspace(nb, cin, cout, h, w, n)
            ws = hip.workspace(wsb, x.device)
            hip.check(_conv_call(lib, "msl_dconv_dgrad", math,
                                 (gy.data_ptr(), packed_d.data_ptr(), dx.data_ptr(), nb, cin, cout, h, w, n, dil0, d1,
                                  ctypes.addressof(ctx.fm), ws.data_ptr(), wsb, s), (gpart,)),
                      "msl_dconv_dgrad")
        sink = grad_sink(weights[0]) if (nb == 1 and not has_bias and ctx.needs_input_grad[1]) else None
        wsb = lib.msl_dconv_wgrad_workspace(nb, cin, cout, h, w, n)
        if sink is not None:
            g, fg, i = sink
            side = _wgrad_stream(x) if ASYNC_WGRAD else None
            with torch.cuda.stream(side) if side is not None else _nullctx():
                ws = hip.workspace(wsb, x.device)
                hip.check(_conv_call(lib, "msl_dconv_wgrad", math,
                                     (x.data_ptr(), gy.data_ptr(), g.data_ptr(), None, 1, cin, cout, h, w, n, dil0, 0, 1,
                                      ctypes.addressof(ctx.fm), ws.data_ptr(), wsb, hip.stream_ptr()), (xpart, gpart)), "msl_dconv_wgrad")
            if side is not None:
                _keep(side, x, gy, *(q[0] for q in (xpart, gpart) if q is not None))
            fg.notify(i)
            return dx, None, None, None, None, None, None, None
        ws = hip.workspace(wsb, x.device)
        dw_all = torch.empty((nb, cout, cin, 3, 3), dtype=_f32, device=x.device)
        db_all = torch.empty((nb, cout), dtype=_f32, device=x.device) if has_bias else None
        hip.check(_conv_call(lib, "msl_dconv_wgrad", math,
                             (x.data_ptr(), gy.data_ptr(), dw_all.data_ptr(), hip.ptr(db_all), nb, cin, cout, h, w,
                              n, dil0, d1, 0, ctypes.addressof(ctx.fm), ws.data_ptr(), wsb, s), (xpart, gpart)), "msl_dconv_wgrad")
        dw0 = dw_all[0]
        dw1 = dw_all[1] if nb > 1 else None
        db0 = db_all[0] if has_bias else None
        db1 = db_all[1] if (has_bias and nb > 1) else None
        return dx, dw0, dw1, db0, db1, None, None, None


def dconv3x3(x, weight, dilation, cache):
    """Stride-1, padding=dilation, bias-free 3x3 conv (Bottleneck.conv2, deeplab_multi.py:17-18)."""
    return _DConv3x3.apply(x, weight, None, None, None, int(dilation), 0, cache)


# --------------------------------------------------------------------------- ASPP heads: shift form
# ASPP_FORM = "shift" (default, r04): the head as one pointwise GEMM with 18*C rows and per-tap shifts
# (csrc/aspp.hip; x read once instead of once per tap), "direct": the two-branch implicit GEMM above.
ASPP_FORM = "shift"


class _ShiftPack:
    """W'[t*C + m][cin] = W_b[m][cin][k] (t = b*9 + k: the head's weights as one pointwise weight) and its
    pointwise packs, rebuilt when a branch weight changes (key: the weights' version counters)."""

    def __init__(self):
        self.key = None
        self.wp = None
        self.pc = PackCache(pointwise=True)
        self.meta = None  # (weights, cin, c) of the last get(): PackBatch refreshes the layout from them

    def get(self, weights, cin, c, for_dgrad):
        self.meta = (list(weights), cin, c)
        self.refresh()
        return self.pc.get([self.wp], cin, 9 * len(weights) * c, for_dgrad)

    def refresh(self):
        """Rebuild W' if a branch weight changed since (its version bump then makes the packs behind it
        stale: PackBatch.run packs them with the step's other packs)."""
        weights, cin, c = self.meta
        key = tuple((w.data_ptr(), w._version) for w in weights)
        nb = len(weights)
        if self.key != key:
            lib = hip.load()
            if self.wp is None or self.wp.shape != (9 * nb * c, cin) or self.wp.device != weights[0].device:
                self.wp = torch.empty((9 * nb * c, cin), dtype=_f32, device=weights[0].device)
            wc = [w.detach().contiguous() for w in weights]
            stride = (wc[1].data_ptr() - wc[0].data_ptr()) // 4 if nb == 2 else 0
            if nb == 2 and (wc[1].data_ptr() - wc[0].data_ptr()) % 4:
                raise hip.MSLError("aspp2: misaligned branch weights")
            hip.check(lib.msl_aspp_weight_layout(wc[0].data_ptr(), stride, nb, c, cin, self.wp.data_ptr(),
                                                 hip.stream_ptr()), "msl_aspp_weight_layout")
            torch.autograd.graph.increment_version(self.wp)  # the packs behind it key on it
            self.key = key


class _ASPPShift(Function):
    """sum_b conv3x3(x, W_b, d_b) + sum_b bias_b as Z = W' x (one pointwise GEMM, M = 18*C) and a
    masked shift-add of Z's rows (msl_aspp_shift_add); backward: G = the shifted, masked copies of dY
    (msl_aspp_shift_gather), dx = W'^T G, dW' = G x^T (the pointwise data / weight gradients)."""

    @staticmethod
    def forward(ctx, x, w0, w1, b0, b1, dil0, dil1, cache):
        ctx.fm = hip.snapshot_forms()  # the backward runs the forms of its forward
        x = _check_act(x, "aspp2", images=True)
        n = _nimg(x)
        weights = [w0] if w1 is None else [w0, w1]
        nb = len(weights)
        c, cin = w0.shape[0], w0.shape[1]
        if w0.shape[2:] != (3, 3) or x.size(1) != cin:
            raise hip.MSLError(f"aspp2: weight {tuple(w0.shape)} does not match input {tuple(x.shape)}")
        h, w = x.shape[-2], x.shape[-1]
        m, p = 9 * nb * c, h * w * n
        lib = hip.load()
        sp = cache.shift_pack()
        packed = sp.get(weights, cin, c, 0)
        z = torch.empty((1, m, p), dtype=_f32, device=x.device)
        wsb = lib.msl_pconv_fwd_workspace(cin, m, p)
        ws = hip.workspace(wsb, x.device)
        math = CONV_MATH
        xpart = _parts(x, math, compute=_split_gemm(m, cin))
        s = hip.stream_ptr()
        hip.check(_conv_call(lib, "msl_pconv_fwd", math,
                             (x.data_ptr(), packed.data_ptr(), z.data_ptr(), cin, m, p,
                              hip.forms(), ws.data_ptr(), wsb, s), (xpart,)), "msl_pconv_fwd")
        bias = None
        if b0 is not None:
            bias = torch.stack([b0] if nb == 1 else [b0, b1]).contiguous()
        y = _like(x, c, h, w)
        hip.check(lib.msl_aspp_shift_add(z.data_ptr(), hip.ptr(bias), y.data_ptr(), nb, c, h, w, n, dil0,
                                         dil1 if nb > 1 else 0, s), "msl_aspp_shift_add")
        ctx.save_for_backward(x, *weights)
        ctx.meta = (nb, cin, c, h, w, n, dil0, dil1, b0 is not None, cache, math)
        ctx.xpart = xpart
        return y

    @staticmethod
    def backward(ctx, gy):
        x, *weights = ctx.saved_tensors
        nb, cin, c, h, w, n, dil0, dil1, has_bias, cache, math = ctx.meta
        gy = gy.contiguous()
        lib = hip.load()
        s = hip.stream_ptr()
        m, p = 9 * nb * c, h * w * n
        g = torch.empty((1, m, p), dtype=_f32, device=x.device)
        db_all = torch.empty((nb, c), dtype=_f32, device=x.device) if has_bias else None
        hip.check(lib.msl_aspp_shift_gather(gy.data_ptr(), g.data_ptr(), hip.ptr(db_all), nb, c, h, w, n, dil0,
                                            dil1 if nb > 1 else 0, s), "msl_aspp_shift_gather")
        gpart = _parts(g, math, compute=True)
        sp = cache.shift_pack()
        dx = None
        if ctx.needs_input_grad[0]:
            packed_d = sp.get(weights, cin, c, 1)
            dx = torch.empty_like(x)
            wsb = lib.msl_pconv_dgrad_workspace(cin, m, p)
            ws = hip.workspace(wsb, x.device)
            cnt = ctypes.addressof(ctx.fm)
            if math == "bf16":
                st = lib.msl_pconv_dgrad_bf16(g.data_ptr(), packed_d.data_ptr(), dx.data_ptr(), cin, m, p, cnt,
                                              ws.data_ptr(), wsb, s)
            else:
                fn = lib.msl_pconv_dgrad_f16 if math == "fp16" else lib.msl_pconv_dgrad_acc_sc
                st = fn(g.data_ptr(), packed_d.data_ptr(), dx.data_ptr(), cin, m, p, 0, cnt, ws.data_ptr(), wsb, s,
                        *_pp(gpart))
            hip.check(st, "msl_pconv_dgrad")
        dw0 = dw1 = None
        if any(ctx.needs_input_grad[1:3]):
            dwp = torch.empty((m, cin), dtype=_f32, device=x.device)
            wsb = lib.msl_pconv_wgrad_workspace(cin, m, p)
            ws = hip.workspace(wsb, x.device)
            hip.check(_conv_call(lib, "msl_pconv_wgrad", math,
                                 (x.data_ptr(), g.data_ptr(), dwp.data_ptr(), cin, m, p, 0, ctypes.addressof(ctx.fm), ws.data_ptr(), wsb, s),
                                 (ctx.xpart, gpart)), "msl_pconv_wgrad")
            dw_all = torch.empty((nb, c, cin, 3, 3), dtype=_f32, device=x.device)
            hip.check(lib.msl_aspp_weight_grad(dwp.data_ptr(), nb, c, cin, dw_all.data_ptr(), s), "msl_aspp_weight_grad")
            dw0 = dw_all[0]
            dw1 = dw_all[1] if nb > 1 else None
        db0 = db_all[0] if has_bias else None
        db1 = db_all[1] if (has_bias and nb > 1) else None
        return dx, dw0, dw1, db0, db1, None, None, None


def aspp2(x, w0, b0, w1, b1, dil0, dil1, cache):
    """conv_d6(x) + conv_d12(x) with biases: the live part of Classifier_Module (deeplab_multi.py:62-66)."""
    if ASPP_FORM == "shift":
        return _ASPPShift.apply(x, w0, w1, b0, b1, int(dil0), int(dil1), cache)
    return _DConv3x3.apply(x, w0, w1, b0, b1, int(dil0), int(dil1), cache)


# --------------------------------------------------------------------------- pointwise conv
class _PConv(Function):
    """y = W x for a 1x1, stride-1, bias-free conv (W: [cout][cin][1][1]) on the HIP pointwise GEMMs:
      y  = W x        msl_pconv_fwd (the conv math's form)
      dx = W^T dy     msl_pconv_dgrad; with a ResidualGrad `hold`, dx = (the identity residual's
                      gradient) + W^T dy, summed by the GEMM's accumulate epilogue (fp32 / fp16)
      dW += dy x^T    msl_pconv_wgrad, straight into the flat gradient buffer when the parameter
                      has a sink
    No library GEMM: every call is deterministic (fixed summation order)."""

    @staticmethod
    def forward(ctx, x, weight, cache, hold=None, grad_to=None):
        ctx.fm = hip.snapshot_forms()  # the backward runs the forms of its forward
        x = _check_act(x, "pconv", images=True)
        cout, cin = weight.shape[0], weight.shape[1]
        if weight.shape[2:] != (1, 1) or x.size(1) != cin:
            raise hip.MSLError(f"pconv: weight {tuple(weight.shape)} does not match input {tuple(x.shape)}")
        h, w = x.shape[-2], x.shape[-1]
        p = h * w * _nimg(x)  # every image: the pixel axis of a pointwise GEMM
        lib = hip.load()
        packed = cache.get([weight], cin, cout, 0)
        y = _like(x, cout, h, w)
        wsb = lib.msl_pconv_fwd_workspace(cin, cout, p)
        ws = hip.workspace(wsb, x.device)
        math = CONV_MATH
        # f16x3: x's absmax partials once for the forward and the weight gradient
        xpart = _parts(x, math, compute=_split_gemm(cout, cin))
        hip.check(_conv_call(lib, "msl_pconv_fwd", math,
                             (x.data_ptr(), packed.data_ptr(), y.data_ptr(), cin, cout, p,
                              hip.forms(), ws.data_ptr(), wsb, hip.stream_ptr()), (xpart,)),
                  "msl_pconv_fwd")
        ctx.save_for_backward(x, weight)
        ctx.meta = (cin, cout, p, cache, math)
        ctx.xpart = xpart
        ctx.hold = hold
        ctx.grad_to = grad_to
        return y

    @staticmethod
    def backward(ctx, gy):
        x, weight = ctx.saved_tensors
        cin, cout, p, cache, math = ctx.meta
        gy = gy.contiguous()
        lib = hip.load()
        s = hip.stream_ptr()
        dx = None
        hold = ctx.hold
        # f16x3: dy's absmax partials once for the data and weight gradients
        gpart = _parts(gy, math, compute=_split_gemm(cin, cout))
        if ctx.needs_input_grad[0]:
            acc = 0
            if hold is not None:
                hold.consumed = True
            res = None
            if hold is not None and hold.g is not None:
                if isinstance(hold.g, MaskedResidual):
                    res, hold.g = hold.g, None
                    if math == "bf16":  # the bf16 form has no epilogue of either kind
                        dx, res, acc = res.materialize(), None, 1
                    else:
                        dx = torch.empty_like(x)
                else:
                    dx, hold.g = hold.g, None
                    acc = 1
            else:
                dx = torch.empty_like(x)
            packed_d = cache.get([weight], cin, cout, 1)
            wsb = lib.msl_pconv_dgrad_workspace(cin, cout, p)
            ws = hip.workspace(wsb, x.device)
            cnt = ctypes.addressof(ctx.fm)
            if math == "bf16":
                tgt = torch.empty_like(x) if acc else dx
                hip.check(lib.msl_pconv_dgrad_bf16(gy.data_ptr(), packed_d.data_ptr(), tgt.data_ptr(), cin, cout, p,
                                                   cnt, ws.data_ptr(), wsb, s), "msl_pconv_dgrad")
                if acc:  # the bf16 form has no accumulate epilogue
                    dx.add_(tgt)
            elif res is not None:  # r06: dx = mask(dy of bn3) + W^T dy, the mask applied in the epilogue
                fn = lib.msl_pconv_dgrad_resmask_f16 if math == "fp16" else lib.msl_pconv_dgrad_resmask_sc
                hip.check(fn(gy.data_ptr(), packed_d.data_ptr(), dx.data_ptr(), cin, cout, p, res.dy.data_ptr(),
                             res.bits.data_ptr(), res.nimg, cnt, ws.data_ptr(), wsb, s, *_pp(gpart)),
                          "msl_pconv_dgrad_resmask")
            else:
                fn = lib.msl_pconv_dgrad_f16 if math == "fp16" else lib.msl_pconv_dgrad_acc_sc
                hip.check(fn(gy.data_ptr(), packed_d.data_ptr(), dx.data_ptr(), cin, cout, p, acc, cnt,
                             ws.data_ptr(), wsb, s, *_pp(gpart)), "msl_pconv_dgrad")
        # a downsample conv (r05): its data gradient goes to the ResidualGrad that the block's conv1 sums
        # into its own (msl_pconv_dgrad_acc) - unless conv1's backward already ran, then autograd adds it
        to = ctx.grad_to
        if dx is not None and to is not None and not to.consumed:
            to.g, dx = dx, None
        if not ctx.needs_input_grad[1]:
            return dx, None, None, None, None
        sink = grad_sink(weight)
        dst = sink[0] if sink is not None else torch.empty_like(weight)
        wsb = lib.msl_pconv_wgrad_workspace(cin, cout, p)
        side = _wgrad_stream(x) if (ASYNC_WGRAD and sink is not None) else None
        with torch.cuda.stream(side) if side is not None else _nullctx():
            ws = hip.workspace(wsb, x.device)
            hip.check(_conv_call(lib, "msl_pconv_wgrad", math,
                                 (x.data_ptr(), gy.data_ptr(), dst.data_ptr(), cin, cout, p, int(sink is not None),
                                  ctypes.addressof(ctx.fm), ws.data_ptr(), wsb, hip.stream_ptr()), (ctx.xpart, gpart)), "msl_pconv_wgrad")
        if side is not None:
            _keep(side, x, gy, *(q[0] for q in (ctx.xpart, gpart) if q is not None))
        if sink is None:
            return dx, dst, None, None, None
        sink[1].notify(sink[2])
        return dx, None, None, None, None


def pconv(x, weight, cache, residual_grad=None, grad_to=None):
    """1x1, stride-1, bias-free conv (Bottleneck.conv1/conv3, downsample: deeplab_multi.py:13,20,96-99).
    `residual_grad` (a ResidualGrad also given to the block's bn_act or downsample conv): its gradient
    is added into this conv's input gradient by the data-gradient GEMM.  `grad_to` (the downsample
    conv of a block, r05): this conv's input gradient is handed to that ResidualGrad instead of to
    autograd, so the block's conv1 sums it (no separate accumulation kernel)."""
    return _PConv.apply(x, weight, cache, residual_grad, grad_to)


conv1x1 = pconv


# --------------------------------------------------------------------------- fused residual gradient
class ResidualGrad:
    """Carries the gradient of a bottleneck's identity residual from bn3's backward (which runs
    first) to conv1's backward, which adds it into the block input's gradient inside its data-
    gradient GEMM (msl_pconv_dgrad_acc) instead of autograd's separate accumulation kernel
    (deeplab_multi.py:31-48: x feeds conv1 and the residual)."""

    __slots__ = ("g", "consumed")

    def __init__(self):
        self.g = None
        self.consumed = False  # the summing conv's backward ran (a later producer hands to autograd)


class MaskedResidual:
    """r06: the identity residual's gradient left unmaterialised - relu'(y) * dy of the block's bn3, as
    bn3's output gradient `dy` and its forward's ReLU mask bits (msl_bn_fwd_mask).  conv1's data-gradient
    GEMM applies the mask in its epilogue (msl_pconv_dgrad_resmask), so bn3's backward skips writing the
    masked copy (one activation-sized write and read per identity block)."""

    __slots__ = ("dy", "bits", "nimg")

    def __init__(self, dy, bits, nimg):
        self.dy, self.bits, self.nimg = dy, bits, nimg

    def materialize(self):
        """The masked gradient as a tensor (the bf16 data-gradient form, which has no epilogue for it)."""
        c, hw = self.dy.size(1), self.dy.size(-2) * self.dy.size(-1)
        words = self.bits.view(c * self.nimg, (hw + 63) // 64)  # [channel][image][word] (msl_bn_relu_mask_bytes)
        idx = torch.arange(hw, device=self.dy.device)
        on = ((words[:, idx // 64] >> (idx % 64)) & 1).bool()  # [channel * image][pixel]
        g = self.dy.reshape(c * self.nimg, hw)  # (1,C[,N],H,W): channel-major, images inside
        return torch.where(on, g, torch.zeros((), dtype=g.dtype, device=g.device)).reshape(self.dy.shape)


# --------------------------------------------------------------------------- stem, maxpool, stride-2 glue
def pool_out(n, k, s, p, ceil):
    """torch's pooling_output_shape (dilation 1)."""
    num = n + 2 * p - (k - 1) - 1 + ((s - 1) if ceil else 0)
    o = num // s + 1
    if ceil and (o - 1) * s >= n + p:
        o -= 1
    return o


class _StemConv(Function):
    """conv2d(x, W, stride, padding) for a bias-free k x k conv as im2col + the pointwise GEMM
    (csrc/stem.hip): the [cout][cin][k][k] weight is a [cout][cin*k*k] pointwise weight as laid out."""

    @staticmethod
    def forward(ctx, x, weight, stride, pad, cache):
        ctx.fm = hip.snapshot_forms()  # the backward runs the forms of its forward
        x = _check_act(x, "stem_conv", images=True)
        cout, cin, kh, kw = weight.shape
        if x.size(1) != cin:
            raise hip.MSLError(f"stem_conv: weight {tuple(weight.shape)} does not match input {tuple(x.shape)}")
        h, w, n = x.shape[-2], x.shape[-1], _nimg(x)
        ho, wo = (h + 2 * pad - kh) // stride + 1, (w + 2 * pad - kw) // stride + 1
        kk, p = cin * kh * kw, ho * wo * n
        lib = hip.load()
        s = hip.stream_ptr()
        col = _like(x, kk, ho, wo)
        hip.check(lib.msl_im2col(x.data_ptr(), cin, h, w, n, kh, kw, stride, pad, 1, ho, wo, col.data_ptr(), s),
                  "msl_im2col")
        wmat = weight.detach().contiguous()
        packed = cache.get([wmat], kk, cout, 0)
        y = _like(x, cout, ho, wo)
        wsb = lib.msl_pconv_fwd_workspace(kk, cout, p)
        ws = hip.workspace(wsb, x.device)
        # the bf16 / fp16 conv maths keep the stem (the raw image, values ~1e2; 2.5 GFLOP per image) in
        # the fp32 form: 8 significant bits there cost 3-4 % of the target loss after one update
        math = "fp32" if CONV_MATH in ("bf16", "fp16") else CONV_MATH
        # f16x3: the column matrix holds the image's values and padding zeros only, and with windows
        # that overlap (stride <= kernel) and reach both borders every pixel is in one: max |col| =
        # max |x|, so the GEMM's operand scale comes from the 3-channel image (r05: a 12-MB pass instead
        # of one over the 147 x P columns, 30-120 us).  The scale is a power of two of that maximum,
        # the same bits either way; the stem's weight gradient (64 x 147, exact-f32 tiles) reads none.
        cover = (stride <= min(kh, kw) and pad < min(kh, kw) and (ho - 1) * stride - pad + kh >= h and
                 (wo - 1) * stride - pad + kw >= w)
        cpart = _parts(x, math) if cover else _parts(col, math, compute=_split_gemm(cout, kk))
        hip.check(_conv_call(lib, "msl_pconv_fwd", math,
                             (col.data_ptr(), packed.data_ptr(), y.data_ptr(), kk, cout, p,
                              hip.forms(), ws.data_ptr(), wsb, s), (cpart,)), "msl_pconv_fwd")
        ctx.save_for_backward(col, weight)
        ctx.meta = (cin, h, w, n, kh, kw, stride, pad, ho, wo, cache, math)
        ctx.cpart = cpart
        return y

    @staticmethod
    def backward(ctx, gy):
        col, weight = ctx.saved_tensors
        cin, h, w, n, kh, kw, stride, pad, ho, wo, cache, math = ctx.meta
        cout, kk, p = weight.shape[0], col.size(1), ho * wo * n
        gy = gy.contiguous()
        lib = hip.load()
        s = hip.stream_ptr()
        dx = None
        gpart = _parts(gy, math, compute=_split_gemm(kk, cout))
        if ctx.needs_input_grad[0]:
            packed_d = cache.get([weight.detach().contiguous()], kk, cout, 1)
            dcol = torch.empty_like(col)
            wsb = lib.msl_pconv_dgrad_workspace(kk, cout, p)
            ws = hip.workspace(wsb, gy.device)
            cnt = ctypes.addressof(ctx.fm)
            if math == "bf16":
                st = lib.msl_pconv_dgrad_bf16(gy.data_ptr(), packed_d.data_ptr(), dcol.data_ptr(), kk, cout, p, cnt,
                                              ws.data_ptr(), wsb, s)
            else:
                fn = lib.msl_pconv_dgrad_f16 if math == "fp16" else lib.msl_pconv_dgrad_acc_sc
                st = fn(gy.data_ptr(), packed_d.data_ptr(), dcol.data_ptr(), kk, cout, p, 0, cnt, ws.data_ptr(), wsb,
                        s, *_pp(gpart))
            hip.check(st, "msl_pconv_dgrad")
            dx = _like(col, cin, h, w)
            hip.check(lib.msl_col2im(dcol.data_ptr(), cin, h, w, n, kh, kw, stride, pad, 1, ho, wo, dx.data_ptr(), s),
                      "msl_col2im")
        if not ctx.needs_input_grad[1]:
            return dx, None, None, None, None
        sink = grad_sink(weight)
        dst = sink[0] if sink is not None else torch.empty_like(weight)
        wsb = lib.msl_pconv_wgrad_workspace(kk, cout, p)
        side = _wgrad_stream(gy) if (ASYNC_WGRAD and sink is not None) else None
        with torch.cuda.stream(side) if side is not None else _nullctx():
            ws = hip.workspace(wsb, gy.device)
            hip.check(_conv_call(lib, "msl_pconv_wgrad", math,
                                 (col.data_ptr(), gy.data_ptr(), dst.data_ptr(), kk, cout, p, int(sink is not None),
                                  ctypes.addressof(ctx.fm), ws.data_ptr(), wsb, hip.stream_ptr()), (ctx.cpart, gpart)), "msl_pconv_wgrad")
        if side is not None:
            _keep(side, col, gy, *(q[0] for q in (ctx.cpart, gpart) if q is not None))
        if sink is None:
            return dx, dst, None, None, None
        sink[1].notify(sink[2])
        return dx, None, None, None, None


def stem_conv(x, weight, stride, pad, cache):
    """nn.Conv2d(cin, cout, k, stride, pad, bias=False) (ResNetMulti.conv1, deeplab_multi.py:73-74)."""
    return _StemConv.apply(x, weight, int(stride), int(pad), cache)


class _MaxPool(Function):
    @staticmethod
    def forward(ctx, x, k, s, p, ceil):
        x = _check_act(x, "maxpool", images=True)
        h, w = x.shape[-2:]
        c = x.size(1) * _nimg(x)  # per plane: every (channel, image)
        ho, wo = pool_out(h, k, s, p, ceil), pool_out(w, k, s, p, ceil)
        y = _like(x, x.size(1), ho, wo)
        idx = _like(x, x.size(1), ho, wo, dtype=torch.int32)
        hip.check(hip.load().msl_maxpool_fwd(x.data_ptr(), c, h, w, k, s, p, ho, wo, y.data_ptr(), idx.data_ptr(),
                                             hip.stream_ptr()), "msl_maxpool_fwd")
        ctx.save_for_backward(idx)
        ctx.meta = (c, h, w, k, s, p, ho, wo)
        ctx.xshape = x.shape
        ctx.mark_non_differentiable(idx)
        return y, idx

    @staticmethod
    def backward(ctx, gy, _gi):
        (idx,) = ctx.saved_tensors
        c, h, w, k, s, p, ho, wo = ctx.meta
        gy = gy.contiguous()
        dx = torch.empty(ctx.xshape, dtype=_f32, device=gy.device)
        hip.check(hip.load().msl_maxpool_bwd(gy.data_ptr(), idx.data_ptr(), c, h, w, k, s, p, ho, wo, dx.data_ptr(),
                                             hip.stream_ptr()), "msl_maxpool_bwd")
        return dx, None, None, None, None


def maxpool2d(x, kernel_size, stride, padding, ceil_mode):
    """nn.MaxPool2d(k, s, p, ceil_mode) (deeplab_multi.py:77); returns the pooled tensor."""
    return _MaxPool.apply(x, int(kernel_size), int(stride), int(padding), bool(ceil_mode))[0]


class _Subsample(Function):
    @staticmethod
    def forward(ctx, x, s):
        x = _check_act(x, "subsample", images=True)
        h, w = x.shape[-2:]
        c = x.size(1) * _nimg(x)  # per plane
        ho, wo = (h - 1) // s + 1, (w - 1) // s + 1
        y = _like(x, x.size(1), ho, wo)
        hip.check(hip.load().msl_subsample(x.data_ptr(), c, h, w, s, ho, wo, y.data_ptr(), hip.stream_ptr()),
                  "msl_subsample")
        ctx.meta = (c, h, w, s, ho, wo)
        ctx.xshape = x.shape
        return y

    @staticmethod
    def backward(ctx, gy):
        c, h, w, s, ho, wo = ctx.meta
        gy = gy.contiguous()
        dx = torch.empty(ctx.xshape, dtype=_f32, device=gy.device)
        hip.check(hip.load().msl_subsample_bwd(gy.data_ptr(), c, h, w, s, ho, wo, dx.data_ptr(), hip.stream_ptr()),
                  "msl_subsample_bwd")
        return dx, None


def subsample(x, stride):
    """x[:, :, ::stride, ::stride] (the input a stride-s 1x1 conv reads)."""
    return _Subsample.apply(x, int(stride))


# --------------------------------------------------------------------------- upsample
class _Upsample(Function):
    @staticmethod
    def forward(ctx, x, ho, wo):
        x = _check_act(x, "upsample")
        c, hi, wi = x.shape[1:]
        y = torch.empty((1, c, ho, wo), dtype=_f32, device=x.device)
        hip.check(hip.load().msl_upsample_fwd(x.data_ptr(), y.data_ptr(), c, hi, wi, ho, wo,
                                              hip.stream_ptr()), "msl_upsample_fwd")
        ctx.meta = (c, hi, wi, ho, wo)
        return y

    @staticmethod
    def backward(ctx, gy):
        c, hi, wi, ho, wo = ctx.meta
        gy = gy.contiguous()
        lib = hip.load()
        gx = torch.empty((1, c, hi, wi), dtype=_f32, device=gy.device)
        wsb = lib.msl_upsample_bwd_workspace(c, hi, wi, ho, wo)
        ws = hip.workspace(wsb, gy.device)
        hip.check(lib.msl_upsample_bwd(gy.data_ptr(), gx.data_ptr(), c, hi, wi, ho, wo, ws.data_ptr(),
                                       wsb, hip.stream_ptr()), "msl_upsample_bwd")
        return gx, None, None


def upsample_bilinear(x, size):
    """F.interpolate(x, size, mode='bilinear', align_corners=True) (deeplab_multi.py:124,128).

    The result carries `_msl_low` = x so the fused losses below can work from
    the low-resolution logits instead of re-reading the upsampled tensor.
    """
    y = _Upsample.apply(x, int(size[0]), int(size[1]))
    y._msl_low = (x, y._version, x._version)
    return y


# --------------------------------------------------------------------------- image pairs
def pair_join(x_s, x_t):
    """(1,C,H,W) x 2 -> the pair (1,C,2,H,W) ([C][2][H][W]) the trunk ops run as one batch."""
    return torch.stack([x_s, x_t], dim=2)


def pair_split(y):
    """(1,C,N,H,W) -> N contiguous (1,C,H,W) images (autograd stacks their gradients back)."""
    return tuple(t.contiguous() for t in y.unbind(2))


# --------------------------------------------------------------------------- fused losses
def _stats(device):
    return torch.empty(hip.load().msl_loss_stats_elems(), dtype=_f32, device=device)


def _geom(low, out_hw):
    c, hi, wi = low.shape[1:]
    return c, hi, wi, int(out_hw[0]), int(out_hw[1])


class _CEUp(Function):
    @staticmethod
    def forward(ctx, low, labels, ho, wo):
        low = _check_act(low, "ce_up")
        labels = labels.contiguous()
        c, hi, wi, ho, wo = _geom(low, (ho, wo))
        if labels.dtype != torch.int64 or labels.numel() != ho * wo:
            raise hip.MSLError(f"ce_up: labels must be int64 with {ho*wo} elements")
        lib = hip.load()
        out = torch.empty((), dtype=_f32, device=low.device)
        st = _stats(low.device)
        wsb = lib.msl_loss_workspace(c, hi, wi, ho, wo)
        ws = hip.workspace(wsb, low.device)
        hip.check(lib.msl_ce_up_fwd(low.data_ptr(), labels.data_ptr(), c, hi, wi, ho, wo, out.data_ptr(),
                                    st.data_ptr(), ws.data_ptr(), wsb, hip.stream_ptr()), "msl_ce_up_fwd")
        ctx.save_for_backward(low, labels, st)
        ctx.geo = (c, hi, wi, ho, wo)
        return out

    @staticmethod
    def backward(ctx, g):
        low, labels, st = ctx.saved_tensors
        c, hi, wi, ho, wo = ctx.geo
        lib = hip.load()
        g = g.to(_f32).contiguous()
        d = torch.empty_like(low)
        wsb = lib.msl_loss_workspace(c, hi, wi, ho, wo)
        ws = hip.workspace(wsb, low.device)
        hip.check(lib.msl_ce_up_bwd(low.data_ptr(), labels.data_ptr(), c, hi, wi, ho, wo, st.data_ptr(),
                                    g.data_ptr(), d.data_ptr(), ws.data_ptr(), wsb, hip.stream_ptr()),
                  "msl_ce_up_bwd")
        return d, None, None, None


class _MaxSquareUp(Function):
    @staticmethod
    def forward(ctx, low, ho, wo):
        low = _check_act(low, "maxsquare_up")
        c, hi, wi, ho, wo = _geom(low, (ho, wo))
        lib = hip.load()
        out = torch.empty((), dtype=_f32, device=low.device)
        st = _stats(low.device)
        wsb = lib.msl_loss_workspace(c, hi, wi, ho, wo)
        ws = hip.workspace(wsb, low.device)
        hip.check(lib.msl_maxsquare_up_fwd(low.data_ptr(), c, hi, wi, ho, wo, out.data_ptr(), st.data_ptr(),
                                           ws.data_ptr(), wsb, hip.stream_ptr()), "msl_maxsquare_up_fwd")
        ctx.save_for_backward(low, st)
        ctx.geo = (c, hi, wi, ho, wo)
        return out

    @staticmethod
    def backward(ctx, g):
        low, st = ctx.saved_tensors
        c, hi, wi, ho, wo = ctx.geo
        lib = hip.load()
        g = g.to(_f32).contiguous()
        d = torch.empty_like(low)
        wsb = lib.msl_loss_workspace(c, hi, wi, ho, wo)
        ws = hip.workspace(wsb, low.device)
        hip.check(lib.msl_maxsquare_up_bwd(low.data_ptr(), c, hi, wi, ho, wo, st.data_ptr(), g.data_ptr(),
                                           d.data_ptr(), ws.data_ptr(), wsb, hip.stream_ptr()),
                  "msl_maxsquare_up_bwd")
        return d, None, None


class _IWMaxSquareUp(Function):
    @staticmethod
    def forward(ctx, low, ho, wo, ratio):
        low = _check_act(low, "iw_maxsquare_up")
        c, hi, wi, ho, wo = _geom(low, (ho, wo))
        lib = hip.load()
        out = torch.empty((), dtype=_f32, device=low.device)
        st = _stats(low.device)
        hist = torch.empty(c, dtype=torch.int32, device=low.device)
        weights = torch.empty(c, dtype=_f32, device=low.device)
        wsb = lib.msl_loss_workspace(c, hi, wi, ho, wo)
        ws = hip.workspace(wsb, low.device)
        hip.check(lib.msl_iw_maxsquare_up_fwd(low.data_ptr(), c, hi, wi, ho, wo, float(ratio), out.data_ptr(),
                                              st.data_ptr(), hist.data_ptr(), weights.data_ptr(), ws.data_ptr(),
                                              wsb, hip.stream_ptr()), "msl_iw_maxsquare_up_fwd")
        ctx.save_for_backward(low, st)
        ctx.geo = (c, hi, wi, ho, wo)
        ctx.mark_non_differentiable(hist, weights)
        return out, hist, weights

    @staticmethod
    def backward(ctx, g, _gh, _gw):
        low, st = ctx.saved_tensors
        c, hi, wi, ho, wo = ctx.geo
        lib = hip.load()
        g = g.to(_f32).contiguous()
        d = torch.empty_like(low)
        wsb = lib.msl_loss_workspace(c, hi, wi, ho, wo)
        ws = hip.workspace(wsb, low.device)
        hip.check(lib.msl_iw_maxsquare_up_bwd(low.data_ptr(), c, hi, wi, ho, wo, st.data_ptr(), g.data_ptr(),
                                              d.data_ptr(), ws.data_ptr(), wsb, hip.stream_ptr()),
                  "msl_iw_maxsquare_up_bwd")
        return d, None, None, None


class _MultiCEUp(Function):
    @staticmethod
    def forward(ctx, low1, low2, ho, wo, thr):
        low1 = _check_act(low1, "multi_ce_up")
        low2 = _check_act(low2.detach(), "multi_ce_up")
        c, hi, wi, ho, wo = _geom(low1, (ho, wo))
        lib = hip.load()
        out = torch.empty((), dtype=_f32, device=low1.device)
        st = _stats(low1.device)
        wsb = lib.msl_loss_workspace(c, hi, wi, ho, wo)
        ws = hip.workspace(wsb, low1.device)
        hip.check(lib.msl_multi_ce_up_fwd(low1.data_ptr(), low2.data_ptr(), c, hi, wi, ho, wo, float(thr),
                                          out.data_ptr(), st.data_ptr(), ws.data_ptr(), wsb, hip.stream_ptr()),
                  "msl_multi_ce_up_fwd")
        ctx.save_for_backward(low1, low2, st)
        ctx.geo = (c, hi, wi, ho, wo, float(thr))
        return out

    @staticmethod
    def backward(ctx, g):
        low1, low2, st = ctx.saved_tensors
        c, hi, wi, ho, wo, thr = ctx.geo
        lib = hip.load()
        g = g.to(_f32).contiguous()
        d = torch.empty_like(low1)
        wsb = lib.msl_loss_workspace(c, hi, wi, ho, wo)
        ws = hip.workspace(wsb, low1.device)
        hip.check(lib.msl_multi_ce_up_bwd(low1.data_ptr(), low2.data_ptr(), c, hi, wi, ho, wo, thr, st.data_ptr(),
                                          g.data_ptr(), d.data_ptr(), ws.data_ptr(), wsb, hip.stream_ptr()),
                  "msl_multi_ce_up_bwd")
        return d, None, None, None, None


def low_of(pred):
    """The low-resolution logits behind an upsampled prediction, or None when there are none or
    when either tensor was modified in place since the upsample (then the loss must read `pred`
    itself: the fused path would silently ignore the edit)."""
    rec = getattr(pred, "_msl_low", None)
    if rec is None:
        return None
    low, v_pred, v_low = rec
    if pred._version != v_pred or low._version != v_low:
        return None
    return low


def loss_labels_up(low1, low2, out_hw, thr=0.95):
    """(argmax, label2) int32 [ho*wo]: the per-pixel decisions of the fused losses - first-max
    argmax of softmax(up(low1)) (IW histogram class) and, if low2 is given, the multi-level
    guidance label with low1 = x1 head, low2 = x2 head (solve_gta5.py:206-212)."""
    low1 = _check_act(low1.detach(), "loss_labels_up")
    c, hi, wi, ho, wo = _geom(low1, out_hw)
    arg = torch.empty(ho * wo, dtype=torch.int32, device=low1.device)
    lab = None
    if low2 is not None:
        low2 = _check_act(low2.detach(), "loss_labels_up")
        lab = torch.empty(ho * wo, dtype=torch.int32, device=low1.device)
    hip.check(hip.load().msl_loss_labels_up(low1.data_ptr(), hip.ptr(low2), c, hi, wi, ho, wo, float(thr),
                                            arg.data_ptr(), hip.ptr(lab), hip.stream_ptr()), "msl_loss_labels_up")
    return arg, lab


def ce_up(low, labels, out_hw):
    return _CEUp.apply(low, labels, int(out_hw[0]), int(out_hw[1]))


def maxsquare_up(low, out_hw):
    return _MaxSquareUp.apply(low, int(out_hw[0]), int(out_hw[1]))


def iw_maxsquare_up(low, out_hw, ratio):
    """Returns (loss, hist int32[C], weights fp32[C])."""
    return _IWMaxSquareUp.apply(low, int(out_hw[0]), int(out_hw[1]), float(ratio))


def multi_ce_up(low1, low2, out_hw, thr):
    return _MultiCEUp.apply(low1, low2, int(out_hw[0]), int(out_hw[1]), float(thr))


# --------------------------------------------------------------------------- prob-input losses
class _MaxSquareProb(Function):
    @staticmethod
    def forward(ctx, prob):
        prob = _check_act(prob, "maxsquare_prob")
        c, hw = prob.size(1), prob.size(2) * prob.size(3)
        lib = hip.load()
        out = torch.empty((), dtype=_f32, device=prob.device)
        wsb = lib.msl_loss_workspace(c, 1, 1, 1, hw)
        ws = hip.workspace(wsb, prob.device)
        hip.check(lib.msl_maxsquare_prob_fwd(prob.data_ptr(), c, hw, out.data_ptr(), ws.data_ptr(), wsb,
                                             hip.stream_ptr()), "msl_maxsquare_prob_fwd")
        ctx.save_for_backward(prob)
        return out

    @staticmethod
    def backward(ctx, g):
        (prob,) = ctx.saved_tensors
        c, hw = prob.size(1), prob.size(2) * prob.size(3)
        g = g.to(_f32).contiguous()
        d = torch.empty_like(prob)
        hip.check(hip.load().msl_maxsquare_prob_bwd(prob.data_ptr(), c, hw, g.data_ptr(), d.data_ptr(),
                                                    hip.stream_ptr()), "msl_maxsquare_prob_bwd")
        return d


class _IWMaxSquareProb(Function):
    @staticmethod
    def forward(ctx, prob, label, ratio):
        prob = _check_act(prob, "iw_maxsquare_prob")
        c, hw = prob.size(1), prob.size(2) * prob.size(3)
        if label is not None:
            label = label.contiguous()
            if label.dtype != torch.int64 or label.numel() != hw:
                raise hip.MSLError("iw_maxsquare_prob: label must be int64 (N,H,W) with N=1")
        lib = hip.load()
        out = torch.empty((), dtype=_f32, device=prob.device)
        hist = torch.empty(c, dtype=torch.int32, device=prob.device)
        weights = torch.empty(c, dtype=_f32, device=prob.device)
        wsb = lib.msl_loss_workspace(c, 1, 1, 1, hw)
        ws = hip.workspace(wsb, prob.device)
        hip.check(lib.msl_iw_maxsquare_prob_fwd(prob.data_ptr(), hip.ptr(label), c, hw, float(ratio),
                                                out.data_ptr(), hist.data_ptr(), weights.data_ptr(),
                                                ws.data_ptr(), wsb, hip.stream_ptr()), "msl_iw_maxsquare_prob_fwd")
        ctx.save_for_backward(prob, weights)
        ctx.mark_non_differentiable(hist, weights)
        return out, hist, weights

    @staticmethod
    def backward(ctx, g, _gh, _gw):
        prob, weights = ctx.saved_tensors
        c, hw = prob.size(1), prob.size(2) * prob.size(3)
        g = g.to(_f32).contiguous()
        d = torch.empty_like(prob)
        hip.check(hip.load().msl_iw_maxsquare_prob_bwd(prob.data_ptr(), c, hw, weights.data_ptr(), g.data_ptr(),
                                                       d.data_ptr(), hip.stream_ptr()), "msl_iw_maxsquare_prob_bwd")
        return d, None, None


def maxsquare_prob(prob):
    return _MaxSquareProb.apply(prob)


def iw_maxsquare_prob(prob, label, ratio):
    return _IWMaxSquareProb.apply(prob, label, float(ratio))


# --------------------------------------------------------------------------- batch norm (+ReLU, +residual)
# r05: the residual BN + ReLU (each bottleneck's bn3, deeplab_multi.py:45-47) keeps its ReLU mask as bits
# for the backward (msl_bn_fwd_mask / msl_bn_bwd_mask) instead of re-reading the block output; the same
# mask bit for bit (tests/test_gpu_ops.py test_bn_relu_mask_bits).  False: the backward reads y.
BN_MASK_BITS = True
RESMASK_DGRAD = True  # r06: MaskedResidual instead of bn3 writing the residual gradient


class _BNAct(Function):
    @staticmethod
    def forward(ctx, x, weight, bias, residual, running_mean, running_var, num_batches, training, momentum,
                eps, relu, hold=None):
        ctx.fm = hip.snapshot_forms()  # the backward runs the forms of its forward
        x = _check_act(x, "bn_act", images=True)
        n = _nimg(x)
        c, p = x.size(1), x.size(-2) * x.size(-1)  # p: pixels of one image
        if residual is not None:
            residual = residual.contiguous()
            if residual.shape != x.shape:
                raise hip.MSLError("bn_act: residual shape mismatch")
        lib = hip.load()
        y = torch.empty_like(x)
        save_mean = torch.empty(c * n, dtype=_f32, device=x.device)
        save_invstd = torch.empty(c * n, dtype=_f32, device=x.device)
        wsb = lib.msl_bn_workspace(c, p, n)
        ws = hip.workspace(wsb, x.device)
        update = bool(training) and running_mean is not None
        # f16x3 / fp16: the per-channel absmax of y for the convs that read it (their operand scales):
        # from registers in the fused kernel, folded into the flat apply otherwise (r05: the big layer1
        # maps of configs 4 / 5 no longer pay a pass of their own)
        fused = bool(lib.msl_bn_uses_fused(c, p, int(bool(training)), hip.forms()))
        am = torch.empty(c, dtype=_f32, device=x.device) if _h3(CONV_MATH) else None
        # r05: a residual BN + ReLU under the fused kernels writes the ReLU mask as bits (msl_bn_fwd_mask),
        # so its backward reads 1 bit per pixel instead of y (msl_bn_bwd_mask)
        bits = None
        if relu and residual is not None and fused and BN_MASK_BITS:
            bits = torch.empty(lib.msl_bn_relu_mask_bytes(c, p, n) // 8, dtype=torch.int64, device=x.device)
        hip.check(lib.msl_bn_fwd_mask(x.data_ptr(), hip.ptr(weight), hip.ptr(bias), hip.ptr(residual), y.data_ptr(),
                                      hip.ptr(running_mean), hip.ptr(running_var), hip.ptr(num_batches),
                                      save_mean.data_ptr(), save_invstd.data_ptr(), c, p, n, int(bool(training)),
                                      int(update), float(momentum), float(eps), int(bool(relu)), hip.forms(),
                                      ws.data_ptr(), wsb, hip.stream_ptr(), hip.ptr(am), hip.ptr(bits)), "msl_bn_fwd")
        if am is not None:
            _tag_absmax(y, am)
        # ReLU without a residual under the fused kernels (p <= 16384): the backward recomputes the
        # mask from x (msl_bn_bwd_am_beta, y = NULL) instead of reading y
        remask = (bool(relu) and residual is None and p <= 16384 and fused)
        ctx.bits = bits
        ctx.save_for_backward(x, weight, y if (relu and not remask and bits is None) else None, save_mean,
                              save_invstd)
        ctx.bias = bias
        ctx.meta = (c, p, n, bool(training), bool(relu))
        ctx.hold = hold
        return y

    @staticmethod
    def backward(ctx, gy):
        x, weight, y, save_mean, save_invstd = ctx.saved_tensors
        c, p, n, training, relu = ctx.meta
        gy = gy.contiguous()
        lib = hip.load()
        nig = ctx.needs_input_grad
        dx = torch.empty_like(x) if nig[0] else None
        hold = ctx.hold
        # r06: an identity block's residual gradient stays unmaterialised (MaskedResidual) when conv1's
        # data-gradient form has the masked epilogue
        lazy = (hold is not None and not nig[3] and ctx.bits is not None and RESMASK_DGRAD and
                CONV_MATH != "bf16" and hasattr(lib, "msl_pconv_dgrad_resmask_sc"))
        dres = torch.empty_like(x) if (nig[3] or (hold is not None and not lazy)) else None
        sw = grad_sink(weight) if nig[1] else None
        sb = grad_sink(ctx.bias) if nig[2] else None
        direct = sw is not None and sb is not None
        if direct:
            dgamma, dbeta = sw[0], sb[0]
        else:
            dgamma = torch.empty(c, dtype=_f32, device=x.device) if nig[1] else None
            dbeta = torch.empty(c, dtype=_f32, device=x.device) if nig[2] else None
        wsb = lib.msl_bn_workspace(c, p, n)
        ws = hip.workspace(wsb, x.device)
        # f16x3 / fp16: the per-channel absmax of dx, the gradient the conv before this BN reads twice
        am = torch.empty(c, dtype=_f32, device=x.device) if (dx is not None and _h3(CONV_MATH)) else None
        if ctx.bits is not None:
            st = lib.msl_bn_bwd_mask(gy.data_ptr(), x.data_ptr(), ctx.bits.data_ptr(), hip.ptr(weight),
                                     hip.ptr(ctx.bias), save_mean.data_ptr(), save_invstd.data_ptr(), hip.ptr(dx),
                                     hip.ptr(dres), hip.ptr(dgamma), hip.ptr(dbeta), c, p, n, int(training), int(relu),
                                     int(direct), ctypes.addressof(ctx.fm), ws.data_ptr(), wsb, hip.stream_ptr(), hip.ptr(am))
        else:
            st = lib.msl_bn_bwd_am_beta(gy.data_ptr(), x.data_ptr(), hip.ptr(y), hip.ptr(weight),
                                        hip.ptr(ctx.bias), save_mean.data_ptr(), save_invstd.data_ptr(),
                                        hip.ptr(dx), hip.ptr(dres), hip.ptr(dgamma), hip.ptr(dbeta), c, p, n,
                                        int(training), int(relu), int(direct), ctypes.addressof(ctx.fm), ws.data_ptr(), wsb,
                                        hip.stream_ptr(), hip.ptr(am))
        hip.check(st, "msl_bn_bwd")
        if am is not None:
            _tag_absmax(dx, am)
        if direct:
            sw[1].notify(sw[2])
            sb[1].notify(sb[2])
            dgamma = dbeta = None
        if hold is not None:  # handed to the block's conv1 backward (ResidualGrad)
            hold.g = MaskedResidual(gy, ctx.bits, n) if lazy else dres
            dres = None
        return dx, dgamma, dbeta, dres, None, None, None, None, None, None, None, None


def bn_act(bn, x, residual=None, relu=False, residual_grad=None):
    """act(bn(x) [+ residual]) for an nn.BatchNorm2d `bn` (train mode: batch statistics, bs = 1).
    With `residual_grad` (ResidualGrad) the residual's gradient goes to that holder instead of
    autograd (pass the residual detached; the conv that shares its input adds it)."""
    training = bn.training or not bn.track_running_stats
    momentum = 0.1 if bn.momentum is None else bn.momentum
    return _BNAct.apply(x, bn.weight, bn.bias, residual, bn.running_mean, bn.running_var,
                        bn.num_batches_tracked if training else None, training, momentum, bn.eps, relu,
                        residual_grad)
