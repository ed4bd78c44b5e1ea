"""SGD with the reference's optimizer semantics, one HIP launch per step.

The reference builds `torch.optim.SGD(params=model.optim_parameters(args),
lr, momentum, weight_decay)` (train_source.py:139-144) from two generator
groups, the first of which lists most backbone parameters 3 or 4 times
(deeplab_multi.py:139-154).  torch's single-tensor SGD
then applies k sequential updates to such a parameter, sharing its momentum
buffer, except that on its first step every occurrence starts a fresh buffer
(the last one is kept).  `SGD` reproduces exactly that, for all parameters of
the model, in a single `msl_sgd_step` launch.

Gradients live in one flat buffer (`FlatGrads`): `param.grad` is a view into
it, `zero_grad()` is one memset, and the data-parallel reducer all-reduces it
in buckets.  A parameter counts as having a gradient this step only if
autograd accumulated into it (post-accumulate-grad hook), so parameters the
reference would leave at `grad=None` (the dead ASPP branches, quirk Q1) are
still skipped, weight decay included.
"""
import numpy as np
import torch

from .. import hip

_ENTRY = np.dtype([("param", "<u8"), ("grad", "<u8"), ("momentum", "<u8"), ("numel", "<i8"),
                   ("mult", "<i4"), ("group", "<i4"), ("has_buf", "<i4"), ("pad", "<i4")])
assert _ENTRY.itemsize == 48


def unique_with_multiplicity(params):
    """[(param, k)] in first-occurrence order; k = number of occurrences (identity)."""
    order, count = [], {}
    for p in params:
        if id(p) not in count:
            count[id(p)] = 0
            order.append(p)
        count[id(p)] += 1
    return [(p, count[id(p)]) for p in order]


class FlatGrads:
    """One flat fp32 gradient buffer; every trainable parameter's .grad is a view of it.

    Parameters are laid out in reverse registration order (the order the
    backward pass produces their gradients), so that contiguous slices of the
    buffer become complete early and can be all-reduced while the backward
    still runs (see utils/dist.py).
    """

    def __init__(self, params, device):
        self.params = list(params)[::-1]
        self.index = {id(p): i for i, p in enumerate(self.params)}
        sizes = [p.numel() for p in self.params]
        self.offsets = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
        self.numel = int(self.offsets[-1])
        self.flat = torch.zeros(self.numel, dtype=torch.float32, device=device)
        self.used = np.zeros(len(self.params), dtype=bool)
        self.listeners = []
        self.gen = 1                                      # backward-pass generation
        self.seen = np.zeros(len(self.params), dtype=np.int64)
        for i, p in enumerate(self.params):
            p.grad = self.flat[self.offsets[i]:self.offsets[i + 1]].view_as(p)
            p.register_post_accumulate_grad_hook(self._make_hook(i))
            # lets the HIP ops accumulate this parameter's gradient in place (ops.grad_sink)
            p._msl_flat = (self, i)

    def _make_hook(self, i):
        def hook(_p):
            self.notify(i)
        return hook

    def notify(self, i):
        """Parameter i's gradient for this backward is complete (AccumulateGrad's hook, or a
        HIP op that accumulated it directly into the flat buffer).  Listeners hear it once per
        backward pass: when an op has accumulated in place and returned None for the parameter,
        autograd still runs the AccumulateGrad node and fires its post-accumulate hook - a second
        report that would count a bucket down before its other parameters are final."""
        self.used[i] = True
        if self.seen[i] == self.gen:
            return
        self.seen[i] = self.gen
        for fn in self.listeners:
            fn(i)

    def new_backward(self):
        """The next reports belong to a new backward pass."""
        self.gen += 1

    def view(self, i):
        return self.flat[self.offsets[i]:self.offsets[i + 1]]

    def zero_(self):
        from .. import ops
        ops.wgrad_join(self.flat.device)  # weight gradients still being accumulated on the side stream
        self.flat.zero_()
        self.used[:] = False
        self.new_backward()

    def reattach(self):
        """Restore the .grad views (e.g. after someone set grads to None)."""
        for i, p in enumerate(self.params):
            if p.grad is None or p.grad.data_ptr() != self.flat.data_ptr() + 4 * int(self.offsets[i]):
                p.grad = self.flat[self.offsets[i]:self.offsets[i + 1]].view_as(p)


class SGD:
    """torch.optim.SGD(params, lr, momentum, weight_decay) for the reference's groups (no nesterov,
    no dampening) - drop-in for train_source.py:139-144."""

    def __init__(self, params, lr, momentum=0.0, weight_decay=0.0, dampening=0.0, nesterov=False):
        if dampening != 0 or nesterov:
            raise NotImplementedError("the reference uses dampening=0, nesterov=False")
        if isinstance(params, torch.Tensor):
            raise TypeError("params must be an iterable of tensors or dicts")
        groups = list(params)
        if groups and not isinstance(groups[0], dict):
            groups = [{"params": groups}]
        self.defaults = dict(lr=lr, momentum=momentum, weight_decay=weight_decay, dampening=0.0, nesterov=False)
        self.param_groups = []
        for g in groups:
            plist = list(g["params"])
            pg = dict(self.defaults)
            pg.update({k: v for k, v in g.items() if k != "params"})
            pg["params"] = plist
            pg["_unique"] = unique_with_multiplicity(plist)
            self.param_groups.append(pg)
        if len(self.param_groups) > 2:
            raise NotImplementedError("at most two parameter groups (backbone, heads)")
        self.state = {}  # param -> {"momentum_buffer": tensor}
        uniq, seen = [], set()
        for g in self.param_groups:
            for p, _ in g["_unique"]:
                if id(p) in seen:
                    raise NotImplementedError("a parameter in two groups")
                seen.add(id(p))
                if p.requires_grad:
                    uniq.append(p)
        self._uniq = uniq
        self.device = uniq[0].device if uniq else torch.device("cpu")
        self.grads = FlatGrads(uniq, self.device)
        self._table_key = None
        self._table = None
        self._last_used = None
        self.grad_scale = 1.0
        self.lr_dev = None  # device float32[2] learning rates (hipGraph replay), else by value

    # -- torch.optim.Optimizer surface ------------------------------------------------
    def zero_grad(self, set_to_none=True):
        """Gradients restart at zero (the flat buffer is cleared; views stay attached)."""
        self.grads.reattach()
        self.grads.zero_()

    def _build_table(self):
        grads = self.grads
        mom = self.defaults["momentum"]
        rows, key = [], []
        for gi, g in enumerate(self.param_groups):
            for p, k in g["_unique"]:
                if not p.requires_grad:
                    continue
                i = grads.index[id(p)]
                if not grads.used[i]:
                    continue  # grad is None in the reference: skipped entirely
                st = self.state.setdefault(p, {})
                has_buf = "momentum_buffer" in st
                if not has_buf:
                    st["momentum_buffer"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                buf = st["momentum_buffer"]
                rows.append((p.data_ptr(), p.grad.data_ptr(), buf.data_ptr(), p.numel(), k, gi, int(has_buf and mom != 0)))
                key.append((rows[-1][0], rows[-1][1], rows[-1][2], rows[-1][6]))
        return rows, tuple(key)

    def prepare(self, used=None):
        """Build (and upload) the launch table for the given live-parameter mask now, creating the
        momentum buffers it needs - so a step captured into a hipGraph afterwards finds it ready
        (no host-to-device copy and no allocation may happen inside the capture).  `used`
        defaults to the parameters that received gradients in the last step."""
        if self._last_used is None:
            raise hip.MSLError("SGD.prepare(): run one step first (its first-step buffer rule, Q2, differs)")
        saved = self.grads.used.copy()
        self.grads.used[:] = self._last_used if used is None else used
        try:
            self._ensure_table()
        finally:
            self.grads.used[:] = saved

    def _ensure_table(self):
        lib = hip.load()
        rows, key = self._build_table()
        if key != self._table_key:
            if torch.cuda.is_current_stream_capturing():
                raise hip.MSLError("SGD: the launch table changed inside a hipGraph capture; call "
                                   "optimizer.prepare() before capturing")
            ent = np.zeros(len(rows), dtype=_ENTRY)
            for j, r in enumerate(rows):
                ent[j] = (r[0], r[1], r[2], r[3], r[4], r[5], r[6], 0)
            numels = ent["numel"].astype(np.int64)
            be = lib.msl_sgd_block_elems()
            nblk_each = (numels + be - 1) // be
            block_entry = np.repeat(np.arange(len(rows), dtype=np.int32), nblk_each)
            starts = np.concatenate([[0], np.cumsum(nblk_each)[:-1]]).astype(np.int64)
            block_offset = (np.arange(int(nblk_each.sum()), dtype=np.int64) - np.repeat(starts, nblk_each)) * be
            blob = np.concatenate([ent.view(np.uint8), block_entry.view(np.uint8), block_offset.view(np.uint8)])
            dev = torch.from_numpy(blob).to(self.device)
            n_ent = ent.nbytes
            n_be = block_entry.nbytes
            self._table = (dev, dev.data_ptr(), dev.data_ptr() + n_ent, dev.data_ptr() + n_ent + n_be,
                           int(nblk_each.sum()))
            self._table_key = key

    def step(self, closure=None):
        if closure is not None:
            raise NotImplementedError("closure")
        if self.device.type != "cuda":
            raise hip.MSLError("SGD.step runs on the HIP path only (no CPU fallback)")
        lib = hip.load()
        from .. import ops
        ops.wgrad_join(self.device)  # the weight gradients accumulated on the side stream (ops.ASYNC_WGRAD)
        self._ensure_table()
        self._last_used = self.grads.used.copy()
        _dev, p_ent, p_be, p_bo, nblocks = self._table
        mom = float(self.defaults["momentum"])
        wd = float(self.defaults["weight_decay"])
        # momentum == 0: buffers are written but has_buf stays 0, i.e. buf = d, p -= lr*d
        if self.lr_dev is not None:
            # learning rates from device memory (set between hipGraph replays, utils/graph.py)
            hip.check(lib.msl_sgd_step_lr_dev(p_ent, p_be, p_bo, nblocks, self.lr_dev.data_ptr(), mom, wd,
                                              float(self.grad_scale), hip.stream_ptr()), "msl_sgd_step_lr_dev")
        else:
            lr0 = float(self.param_groups[0]["lr"])
            lr1 = float(self.param_groups[1]["lr"]) if len(self.param_groups) > 1 else lr0
            hip.check(lib.msl_sgd_step(p_ent, p_be, p_bo, nblocks, lr0, lr1, mom, wd, float(self.grad_scale),
                                       hip.stream_ptr()), "msl_sgd_step")
        # the kernel wrote the parameters behind autograd's back: bump their version counters
        for g in self.param_groups:
            for p, _ in g["_unique"]:
                if p.requires_grad and self.grads.used[self.grads.index[id(p)]]:
                    torch.autograd.graph.increment_version(p)
        return None

    def group_lrs(self):
        lr0 = float(self.param_groups[0]["lr"])
        return lr0, (float(self.param_groups[1]["lr"]) if len(self.param_groups) > 1 else lr0)

    # -- checkpoints (train_source.py:662-704 stores optimizer.state_dict()) -----------
    def state_dict(self):
        """torch.optim.Optimizer.state_dict's format: list positions numbered across the groups,
        every occurrence of a duplicated parameter (Q2) mapped to one position, and one
        momentum buffer per tensor under that index - what the reference's torch.optim.SGD writes
        into its checkpoints (train_source.py:672-674)."""
        first, start, groups = {}, 0, []
        for g in self.param_groups:
            # torch's pack_group: one dict comprehension per group, so inside a group the LAST
            # position of a duplicated tensor wins; a tensor seen in an earlier group keeps that one
            first.update({id(p): i for i, p in enumerate(g["params"], start) if id(p) not in first})
            pg = {k: v for k, v in g.items() if k not in ("params", "_unique")}
            pg["params"] = [first[id(p)] for p in g["params"]]
            start += len(g["params"])
            groups.append(pg)
        state = {}
        for g in self.param_groups:
            for p, _ in g["_unique"]:
                st = self.state.get(p)
                if st is not None and "momentum_buffer" in st:
                    state[first[id(p)]] = {"momentum_buffer": st["momentum_buffer"].detach().clone()}
        return {"state": state, "param_groups": groups}

    def load_state_dict(self, sd):
        """Accepts this class's and torch.optim.SGD's state dicts (same format)."""
        flat = [p for g in self.param_groups for p in g["params"]]
        for i, s in sd["state"].items():
            p = flat[int(i)]
            if "momentum_buffer" in s:
                self.state.setdefault(p, {})["momentum_buffer"] = s["momentum_buffer"].to(p.device).clone()
        for g, sg in zip(self.param_groups, sd["param_groups"]):
            for k, v in sg.items():
                if k in ("lr", "momentum", "weight_decay"):
                    g[k] = v
        self._table_key = None
