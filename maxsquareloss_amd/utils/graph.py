"""One training iteration as a hipGraph (torch.cuda.CUDAGraph on ROCm).

A bs=1 UDA iteration (solve_gta5.py:335-387) is ~1,600 kernel launches with static shapes;
enqueued eagerly from Python it costs the host ~35 ms per iteration, which bounds the step once
the kernels are faster than that (profiles/r01_host_bound.txt).  `GraphedStep` runs the first
iteration eagerly on its own stream - that settles the caching allocator, the MIOpen / hipBLASLt
handles, the SGD launch table with the reference's first-step momentum rule (quirk Q2) and the
live parameter set - then captures the iteration body once and replays it for every later
iteration:
  - inputs are copied into the captured (static) buffers before each replay;
  - the poly learning rates (train_source.py:706-717) change every iteration: the captured SGD
    kernel reads them from device memory (msl_sgd_step_lr_dev), refreshed from a pinned host
    ring before each replay;
  - every weight pack (ops.PackCache) and the SGD step are inside the graph, so each replay
    repacks from the weights the previous replay updated; after a replay the parameters'
    version counters are bumped so eager code outside the graph repacks too;
  - loss scalars / meters are the captured tensors, rewritten in place by every replay.
Data-parallel runs (a GradReducer with host-driven bucket countdown) stay eager.
"""
import torch


class GraphedStep:
    def __init__(self, trainer, body, ring=4):
        self.tr = trainer
        self.body = body
        self.graph = None
        self.static = None
        self.device = trainer.device
        self.stream = torch.cuda.Stream(device=self.device)
        self.lr_dev = torch.zeros(2, dtype=torch.float32, device=self.device)
        self.ring = [torch.zeros(2, dtype=torch.float32).pin_memory() for _ in range(ring)]
        self.ring_ev = [None] * ring
        self.k = 0
        self.replays = 0

    def _set_lr(self):
        slot = self.k % len(self.ring)
        self.k += 1
        ev = self.ring_ev[slot]
        if ev is not None:
            ev.synchronize()  # the copy that last read this slot is done (only waits if far behind)
        lr0, lr1 = self.tr.optimizer.group_lrs()
        self.ring[slot][0] = lr0
        self.ring[slot][1] = lr1
        self.lr_dev.copy_(self.ring[slot], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self.ring_ev[slot] = ev

    def __call__(self, *inputs):
        if self.graph is None:
            self._first(*inputs)
            return
        for s, x in zip(self.static, inputs):
            if s.data_ptr() != x.data_ptr():
                s.copy_(x, non_blocking=True)
        self._set_lr()
        self.graph.replay()
        self.replays += 1
        opt = self.tr.optimizer
        for p in opt._uniq:
            torch.autograd.graph.increment_version(p)

    def _first(self, *inputs):
        opt = self.tr.optimizer
        self.static = [x.detach().clone() for x in inputs]
        s = self.stream
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            self.body(*self.static)  # iteration 0, eager (host learning rates)
        torch.cuda.current_stream(self.device).wait_stream(s)
        opt.prepare()  # the table of every later step (buffers exist: has_buf = 1)
        opt.lr_dev = self.lr_dev
        owners = [self.tr] + [m for m in vars(self.tr).values() if isinstance(m, torch.nn.Module)]
        before = [{k: v for k, v in vars(o).items() if isinstance(v, torch.Tensor)} for o in owners]
        try:
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph, stream=s):
                self.body(*self.static)
        finally:
            opt.lr_dev = None  # eager steps outside the graph keep passing the rates by value
        # the capture rebound the step's outputs (loss scalars, IW histogram, ...) to tensors the
        # graph writes but has not written yet: give them iteration 0's values
        with torch.cuda.stream(s):
            for o, old in zip(owners, before):
                for k, v in old.items():
                    new = getattr(o, k, None)
                    if isinstance(new, torch.Tensor) and new is not v and new.shape == v.shape:
                        new.copy_(v)
        torch.cuda.current_stream(self.device).wait_stream(s)
