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
    version counters are bumped so eager code outside the graph repacks too, and recorded: a
    parameter changed eagerly between replays (load_checkpoint, an in-place edit) shows as a new
    version, and the packs are then rebuilt eagerly before the next replay reads them;
  - loss scalars / meters are the captured tensors, rewritten in place by every replay.
Data-parallel runs (a GradReducer, whose bucket countdown is host-driven) capture the
forward/backward passes (the reducer deferred) and the update (`update`: SGD, zero_grad, packs) as
separate graphs.  The passes may be captured as several consecutive `segments` (r04, pair mode: the
backward split at layer3's output) with a host call after each (`between`): each iteration replays
segment 1, launches the exchange of the gradients it finished on RCCL's stream, replays segment 2
meanwhile, launches the rest and joins it, then replays the update.  Those captures use the
thread-local capture mode, so RCCL's / gloo's own threads may keep calling the HIP runtime meanwhile.
"""
import gc
import torch


class GraphedStep:
    def __init__(self, trainer, body, ring=4, exchange=None, update=None, segments=None, between=None):
        self.tr = trainer
        self.body = body
        self.exchange = exchange
        self.update = update
        # the captured passes: segments[0](*inputs), segments[1](), ...; between[i]() runs after the
        # replay of segment i (data parallel: the exchange)
        self.segments = segments if segments is not None else [body]
        self.between = between if between is not None else ([exchange] if exchange is not None else [])
        self.graph = None
        self.graphs = []
        self.graph_update = None
        self.static = None
        self.device = trainer.device
        self.stream = torch.cuda.Stream(device=self.device)
        self.lr_dev = torch.zeros(2, dtype=torch.float32, device=self.device)
        self.ring = [torch.zeros(2, dtype=torch.float32).pin_memory() for _ in range(ring)]
        self.ring_ev = [None] * ring
        self.k = 0
        self.replays = 0
        self.versions = None   # the parameters' versions right after the last replay's bump
        self.eager_repacks = 0

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
        opt = self.tr.optimizer
        if self.versions is not None and any(p._version != v for p, v in zip(opt._uniq, self.versions)):
            # weights edited outside the graph since the last replay: its captured forward reads the
            # packs the last replay wrote, so rebuild them from the current weights first
            self.tr.packer.run()
            self.eager_repacks += 1
        self._set_lr()
        for i, g in enumerate(self.graphs):
            g.replay()
            if i < len(self.between):
                self.between[i]()
        if self.graph_update is not None:
            self.graph_update.replay()
        self.replays += 1
        for p in opt._uniq:
            torch.autograd.graph.increment_version(p)
        self.versions = [p._version for p in opt._uniq]

    def _first(self, *inputs):
        opt = self.tr.optimizer
        self.static = [x.detach().clone() for x in inputs]
        s = self.stream
        s.wait_stream(torch.cuda.current_stream(self.device))
        dp = self.update is not None  # data parallel: the update is a graph of its own
        red = self.tr.reducer if dp else None
        with torch.cuda.stream(s):
            if dp:  # iteration 0, eager, with the overlapped exchange (learns the live set)
                self.body(*self.static)
                red.finish()
                self.update()
            else:
                self.body(*self.static)  # iteration 0, eager (host learning rates)
        torch.cuda.current_stream(self.device).wait_stream(s)
        torch.cuda.synchronize(self.device)
        opt.prepare()  # the table of every later step (buffers exist: has_buf = 1)
        opt.lr_dev = self.lr_dev
        owners = [self.tr] + [m for m in vars(self.tr).values() if isinstance(m, torch.nn.Module)]
        before = [{k: v for k, v in vars(o).items() if isinstance(v, torch.Tensor)} for o in owners]
        mode = "thread_local" if dp else "global"
        # no Python garbage collection while a stream captures: a collected CUDA graph or event of an
        # earlier trainer (reference cycles) would call the runtime from its destructor, which a capturing
        # stream forbids (hipErrorStreamCaptureUnsupported, an abort; found on RCCL, r05).  torch.cuda.graph
        # collects once on entry.
        gc_was = gc.isenabled()
        gc.disable()
        try:
            if dp:
                red.deferred = True
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph, stream=s, capture_error_mode=mode):
                self.segments[0](*self.static)
            self.graphs = [self.graph]
            for seg in self.segments[1:]:  # later segments read the first one's tensors: one memory pool
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, pool=self.graph.pool(), stream=s, capture_error_mode=mode):
                    seg()
                self.graphs.append(g)
            if dp:
                self.graph_update = torch.cuda.CUDAGraph()
                with torch.cuda.graph(self.graph_update, stream=s, capture_error_mode=mode):
                    self.update()
        finally:
            if gc_was:
                gc.enable()
            opt.lr_dev = None  # eager steps outside the graph keep passing the rates by value
            if dp:
                red.deferred = False
        # the capture rebound the step's outputs (loss scalars, IW histogram, ...) to tensors the
        # graph writes but has not written yet: give them iteration 0's values
        with torch.cuda.stream(s):
            for o, old in zip(owners, before):
                for k, v in old.items():
                    new = getattr(o, k, None)
                    if isinstance(new, torch.Tensor) and new is not v and new.shape == v.shape:
                        new.copy_(v)
        torch.cuda.current_stream(self.device).wait_stream(s)
        #  the packs the captured forward reads were built from these versions: an eager
        # weight edit before the first replay must trigger the same repack as one between replays
        self.versions = [p._version for p in opt._uniq]
