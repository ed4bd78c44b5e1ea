"""Data-parallel gradient exchange: bucketed all-reduce overlapped with the backward.

The reference has no torch.distributed at all; its only
"parallelism" is a one-device nn.DataParallel.  The MI355X step runs one
process per GPU (bs = 1 image per rank and per domain, BN per replica, Q9)
and exchanges exactly one thing per iteration: the gradient sum of the live
parameters (43.55 M fp32).  Over xGMI that is an RCCL ring all-reduce
(backend "nccl" on ROCm); on CPU tests the same code runs on gloo.

Overlap: gradients sit in one flat buffer laid out in backward order
(utils/optim.FlatGrads).  Before the LAST backward of an iteration (the target
backward; the source backward only accumulates locally) the reducer is armed;
each post-accumulate-grad hook counts down its bucket, and a bucket whose live
parameters are all final is all-reduced immediately, asynchronously, on RCCL's
own stream (ProcessGroupNCCL orders it after the producing kernels with an
event), while autograd keeps issuing backward kernels on the compute stream.
Buckets launch strictly in index order so every rank issues the same
collective sequence.  `finish()` makes the compute stream wait for the last
bucket; the averaging 1/world is folded into the SGD kernel (grad_scale).

Dead parameters (Q1: ASPP branches d=18/24, or layer5 when --multi False)
never fire a hook; they are discovered on the first iteration and excluded.

Captured steps (utils/graph.py, --graph): the bucket countdown is host-driven, so a replayed graph
cannot launch collectives from inside the backward.  There the reducer is `deferred` while the
iteration is captured (no hook launches anything) and the backward is captured as two graphs, split at
layer3's output (r04): the first (forward + the backward through the heads and layer4) leaves the
gradients of the first `n_early` parameters in backward order final, and `reduce_early()` all-reduces
the buckets made of those alone on RCCL's stream while the next graph replays on the compute stream.
r05: the backward is also cut inside layer3 (the model's split_cuts); after each further segment
`reduce_more()` launches the buckets it finished (bucket bounds end at every segment's end,
`set_breaks`), and `reduce_rest()` launches the rest after the last segment and joins the exchange
before the SGD graph: 88 % of the live gradient bytes are launched before the last segment (layer3.0-2,
layer2, layer1, the stem) replays.  Without a split (two-pass mode) `reduce_all()` exchanges every
bucket after the backward.
"""
import numpy as np
import torch
import torch.distributed as dist


class GradReducer:
    def __init__(self, optimizer, bucket_cap_mb=25.0, process_group=None, always=False):
        self.opt = optimizer
        self.flat = optimizer.grads
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if dist.is_initialized() else 1
        # always: launch the collectives at one rank too (--dp_exchange: the RCCL path on one GPU)
        self.always = bool(always) and dist.is_initialized()
        self.cap = int(bucket_cap_mb * 1024 * 1024 / 4)
        self.set_breaks([])
        self.live = None        # bool mask of parameters that receive gradients
        self.armed = False
        self.works = []
        self.deferred = False   # True while a graph captures the backward (utils/graph.py)
        self.flat.listeners.append(self._on_grad)
        optimizer.grad_scale = 1.0 / self.world

    def set_breaks(self, breaks):
        """Buckets = contiguous parameter ranges of ~cap elements in flat (backward) order that also
        end at every index in `breaks` (the parameter counts a split backward's segments finish, so no
        bucket waits for a later segment)."""
        ends = set(int(b) for b in breaks)
        self.bucket_of = np.zeros(len(self.flat.params), dtype=np.int64)
        bounds, start_p, acc = [], 0, 0
        for i, p in enumerate(self.flat.params):
            acc += p.numel()
            self.bucket_of[i] = len(bounds)
            if acc >= self.cap or (i + 1) in ends:
                bounds.append((start_p, i + 1))
                start_p, acc = i + 1, 0
        if start_p < len(self.flat.params):
            bounds.append((start_p, len(self.flat.params)))
        self.bounds = bounds
        if getattr(self, "live", None) is not None:
            self.has_live = [bool(self.live[lo:hi].any()) for lo, hi in self.bounds]

    def _elem_range(self, b):
        lo, hi = self.bounds[b]
        return int(self.flat.offsets[lo]), int(self.flat.offsets[hi])

    def _launch(self, b):
        a, e = self._elem_range(b)
        if self.world > 1 or self.always:
            from .. import ops
            ops.wgrad_join(self.flat.flat.device)  # the bucket's weight gradients may be on the side stream
            self.works.append(dist.all_reduce(self.flat.flat[a:e], group=self.pg, async_op=True))

    def _advance(self):
        while self.next < len(self.bounds) and self.pending[self.next] == 0:
            if self.has_live[self.next]:
                self._launch(self.next)
            self.next += 1

    def prepare_for_backward(self):
        """Call right before the last backward of the iteration."""
        self.works = []
        self.flat.new_backward()
        if self.live is None or self.deferred:
            self.armed = False
            return
        self.pending = [int(self.live[lo:hi].sum()) for lo, hi in self.bounds]
        self.has_live = [p > 0 for p in self.pending]
        self.next = 0
        self.armed = True
        self._advance()

    def _on_grad(self, i):
        if not self.armed or not self.live[i]:
            return
        b = int(self.bucket_of[i])
        self.pending[b] -= 1
        if self.pending[b] == 0:
            self._advance()

    def finish(self):
        """Complete the exchange; afterwards the flat buffer holds the rank-sum of gradients."""
        if self.live is None:
            # first iteration: learn the live set (identical on every rank), reduce everything now
            self.live = self.flat.used.copy()
            self.pending = [0] * len(self.bounds)
            self.has_live = [bool(self.live[lo:hi].any()) for lo, hi in self.bounds]
            self.next = 0
            self.works = []
            self._advance()
        elif self.armed:
            if self.next < len(self.bounds):
                # a bucket never completed in the armed backward (its params only got grads earlier)
                for b in range(self.next, len(self.bounds)):
                    self.pending[b] = 0
                self._advance()
        for w in self.works:
            w.wait()
        self.works = []
        self.armed = False

    def reduce_early(self, n_early):
        """Launch (asynchronously, on RCCL's stream) every live bucket made only of the first `n_early`
        parameters in backward order - final after the first segment of a split backward."""
        if self.live is None:
            raise RuntimeError("GradReducer.reduce_early before the live set is known (run one eager step)")
        self.works = []
        self.next = 0
        while self.next < len(self.bounds) and self.bounds[self.next][1] <= n_early:
            if self.has_live[self.next]:
                self._launch(self.next)
            self.next += 1

    def reduce_more(self, n_final):
        """reduce_early's continuation after a later segment: launch the next live buckets made only
        of the first `n_final` parameters."""
        while self.next < len(self.bounds) and self.bounds[self.next][1] <= n_final:
            if self.has_live[self.next]:
                self._launch(self.next)
            self.next += 1

    def reduce_rest(self):
        """Launch the buckets reduce_early left and make the current stream wait for every bucket."""
        for b in range(self.next, len(self.bounds)):
            if self.has_live[b]:
                self._launch(b)
        self.next = len(self.bounds)
        for w in self.works:
            w.wait()
        self.works = []

    def reduce_all(self):
        """All-reduce every live bucket now (a replayed step: the backward ran inside a graph) and
        make the current stream wait for the result."""
        if self.live is None:
            raise RuntimeError("GradReducer.reduce_all before the live set is known (run one eager step)")
        self.works = []
        for b in range(len(self.bounds)):
            if self.has_live[b]:
                self._launch(b)
        for w in self.works:
            w.wait()
        self.works = []
