"""CPU tests of the host side: the C-ABI library, the model/optimizer plumbing and DP exchange."""
import ctypes
import json
import os
import re
import socket
import subprocess
import sys
from collections import Counter

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")


def _header_symbols():
    src = open(os.path.join(ROOT, "include", "msl_hip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(msl_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    from maxsquareloss_amd import hip
    lib = hip.load(require_gpu=False)
    syms = _header_symbols()
    assert len(syms) >= 30
    for s in syms:
        assert hasattr(lib, s), s
    assert set(hip.SIGNATURES) == set(syms), "ctypes signatures out of sync with include/msl_hip.h"
    out = subprocess.run(["nm", "-D", "--defined-only", hip.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (msl_\w+)", out))
    assert set(syms) <= exported


def test_every_launch_is_guarded():
    """every kernel launch in csrc/ goes through MSL_LAUNCH, which checks the block
    against the kernel's __launch_bounds__ on the host and returns MSL_ERR_LAUNCH instead of launching
    (tests/test_gpu_ops.py::test_launch_guard_refuses_oversized_blocks runs it on the GPU)."""
    csrc = os.path.join(ROOT, "maxsquareloss_amd", "csrc")
    n = 0
    for f in sorted(os.listdir(csrc)):
        if f.endswith(".hip"):
            src = open(os.path.join(csrc, f)).read()
            assert "hipLaunchKernelGGL" not in src, f
            n += src.count("MSL_LAUNCH(")
    assert n >= 80
    internal = open(os.path.join(csrc, "msl_internal.h")).read()
    assert internal.count("hipLaunchKernelGGL") == 1 and "launch_guard" in internal


@pytest.mark.parametrize("H,W,C", [(512, 1024, 19), (640, 1280, 19), (760, 1280, 16), (380, 640, 16)])
def test_f16_wgrad_predicate_matches_library(H, W, C):
    """the fp16 envelope's weight-gradient rounding predicate is the oracle's restatement
    of the design rule (orc.f16_wgrad_rounds), and it equals the library's own plan (msl_conv_wgrad_split,
    a pure-host query) on every conv of the model at the config sizes (configs[1..4], the fp16 loss-curve
    size 640 x 380) - so a wrong plan in the library is caught instead of mirrored."""
    from oracle import msl_oracle as orc
    from maxsquareloss_amd import hip
    lib = hip.load(require_gpu=False)
    calls = orc.conv_calls(H, W, C)
    assert len(calls) == 107  # 33 bottlenecks x 3 + 4 downsamples (the stem excluded) + 2 heads x 2 live branches
    pred = orc.f16_wgrad_rounds(C)
    n_round = 0
    for cin, cout, k, h, w in sorted(set(calls)):
        if k == 3 and cout == C:
            lib_r = lib.msl_conv_wgrad_split(1, 1, cin, 18 * C, h, w, 2)
        else:
            lib_r = lib.msl_conv_wgrad_split(1, 9 if k == 3 else 1, cin, cout, h, w, 2)
        assert lib_r in (0, 1)
        assert pred(cin, cout, k, h, w) == bool(lib_r), (cin, cout, k, h, w)
        n_round += lib_r
    assert 10 <= n_round <= 21  # most wide convs round; layer1's 64-channel ones never do


def test_library_is_gfx950_code_object():
    import shutil
    import tempfile
    from maxsquareloss_amd import hip
    # (llvm-objdump --offloading extracts the bundles next to its input: work on a copy outside the tree)
    with tempfile.TemporaryDirectory() as d:
        lib = shutil.copy(hip.LIB_PATH, d)
        out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", lib],
                             capture_output=True, text=True, cwd=d)
    assert "gfx950" in (out.stdout + out.stderr)


def test_pure_host_entry_points():
    from maxsquareloss_amd import hip
    lib = hip.load(require_gpu=False)
    assert lib.msl_abi_version() == hip.ABI_VERSION
    assert lib.msl_status_string(-2) == b"workspace too small"
    assert lib.msl_status_string(-4) == b"block exceeds the kernel's launch bounds"
    # packed-weight sizes: [nbranch][ceil(cimg/16)][9][16] rows x round_up(m, 128), x 2.5 for the
    # planes, + the 320-float tail (the f16x3 form's weight absmax partials and scale)
    assert lib.msl_dconv_packed_elems(1, 256, 256, 0) == 16 * 9 * 16 * 256 * 5 // 2 + 320
    assert lib.msl_dconv_packed_elems(2, 2048, 19, 0) == 2 * 128 * 9 * 16 * 128 * 5 // 2 + 320
    assert lib.msl_dconv_packed_elems(2, 2048, 19, 1) == 2 * 2 * 9 * 16 * 2048 * 5 // 2 + 320
    assert lib.msl_dconv_fwd_workspace(1, 256, 256, 65, 129, 1) > 0  # split-K slabs at this size
    assert lib.msl_loss_stats_elems() == 64
    be = lib.msl_sgd_block_elems()
    numels = np.array([10, be, be + 1, 0], dtype=np.int64)
    assert lib.msl_sgd_plan(numels.ctypes.data, 4, None, None, 0) == 1 + 1 + 2
    ent = np.zeros(8, np.int32)
    off = np.zeros(8, np.int64)
    n = lib.msl_sgd_plan(numels.ctypes.data, 4, ent.ctypes.data, off.ctypes.data, 8)
    assert n == 4 and list(ent[:4]) == [0, 1, 2, 2] and list(off[:4]) == [0, 0, 0, be]
    # the per-call kernel forms (ABI 3, msl_forms): defaults f16x3 (5), hybrid schedule, one-launch
    # packs, fused BN; f32 MFMA (0) and bf16x6 (2) selectable, other values refused; NULL = defaults
    d = hip.Forms()
    assert lib.msl_forms_default(ctypes.addressof(d)) == 0
    assert (d.f32_form, d.sk_hybrid, d.pack_form, d.bn_fused) == (5, 1, 1, 1)
    assert [(f, getattr(hip.FORMS, f)) for f, _ in hip.Forms._fields_] == [(f, getattr(d, f)) for f, _ in d._fields_]
    assert lib.msl_forms_check(None) == 0
    for field, good, bad in (("f32_form", (0, 2, 5), (1, 7, -1)), ("sk_hybrid", (0, 1), (2,)),
                             ("pack_form", (0, 1), (2,)), ("bn_fused", (0, 1), (2, -1))):
        for v in good + bad:
            t = hip.Forms(5, 1, 1, 1)
            setattr(t, field, v)
            assert lib.msl_forms_check(ctypes.addressof(t)) == (0 if v in good else -3), (field, v)
    t = hip.Forms(5, 1, 1, 2)
    assert lib.msl_bn_uses_fused(256, 8385, 1, ctypes.addressof(t)) == -3
    assert lib.msl_bn_uses_fused(256, 8385, 1, None) == 1
    t.bn_fused = 0
    assert lib.msl_bn_uses_fused(256, 8385, 1, ctypes.addressof(t)) == 0
    # hip.set_form checks before it sets and returns the previous value
    assert hip.set_form("sk_hybrid", 0) == 1 and hip.FORMS.sk_hybrid == 0
    assert hip.set_form("sk_hybrid", 1) == 0
    with pytest.raises(hip.MSLError):
        hip.set_form("f32_form", 3)
    assert hip.FORMS.f32_form == 5


def test_compute_calls_fail_loudly_without_gpu():
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from maxsquareloss_amd import hip, ops
    with pytest.raises(hip.MSLError):
        ops.dconv3x3(torch.zeros(1, 4, 5, 5), torch.zeros(4, 4, 3, 3), 2, ops.PackCache())
    with pytest.raises(hip.MSLError):
        hip.load(require_gpu=True)


def test_model_matches_reference_structure():
    from oracle import msl_oracle as orc
    from maxsquareloss_amd.graphs.models.deeplab_multi import DeeplabMulti
    m = DeeplabMulti(19, pretrained=False)
    specs = orc.param_specs(19)
    assert [n for n, _ in m.named_parameters()] == [n for n, _, _ in specs]
    assert [tuple(p.shape) for _, p in m.named_parameters()] == [s for _, s, _ in specs]
    assert sum(p.numel() for p in m.parameters()) == 44601560
    assert not m.bn1.weight.requires_grad
    with pytest.raises(FileNotFoundError):
        DeeplabMulti(19, pretrained=True)


def test_optim_parameters_duplicates_match_reference():
    from maxsquareloss_amd.graphs.models.deeplab_multi import DeeplabMulti
    from maxsquareloss_amd.utils.optim import unique_with_multiplicity
    m = DeeplabMulti(19, pretrained=False)
    names = {id(p): n for n, p in m.named_parameters()}

    class A:
        lr = 2.5e-4
    groups = m.optim_parameters(A)
    lists = [[names[id(p)] for p in g["params"]] for g in groups]
    ref = json.load(open(os.path.join(GOLD, "optim_lists.json")))
    assert lists[0] == ref["group0"] and lists[1] == ref["group1"]
    groups = m.optim_parameters(A)
    uniq = unique_with_multiplicity(list(groups[0]["params"]))
    mult = Counter(k for _, k in uniq)
    assert mult == Counter({3: 297, 4: 12, 1: 1})
    live = sum(p.numel() for n, p in m.named_parameters()
               if p.requires_grad and not any(f"conv2d_list.{i}" in n for i in (2, 3)))
    assert live == 43550732  # the live fp32 gradient set exchanged per iteration


def test_synthetic_generators_are_deterministic():
    from maxsquareloss_amd.utils.synthetic import counter_normal, synthetic_image, synthetic_labels
    a = counter_normal(1, "x", 1000, 0.01)
    assert np.array_equal(a, counter_normal(1, "x", 1000, 0.01))
    assert abs(a.std() - 0.01) < 0.001 and abs(a.mean()) < 0.002
    img = synthetic_image(8, 16, 3)
    assert img.shape == (1, 3, 8, 16) and img.dtype == torch.float32
    assert img.min() >= -123 and img.max() <= 256 - 104
    lab = synthetic_labels(8, 16, 19, 3)
    assert lab.dtype == torch.int64 and lab.min() >= -1 and lab.max() <= 18


def test_bench_feature_geometry():
    sys.path.insert(0, ROOT)
    import bench
    assert bench.feat_hw(512) == 65 and bench.feat_hw(1024) == 129
    assert bench.feat_hw(640) == 81 and bench.feat_hw(760) == 96 and bench.feat_hw(1280) == 161


def test_model_runs_no_library_conv():
    """Every conv / pool module of DeeplabMulti forwards to the HIP kernels (no MIOpen / hipBLASLt /
    ATen pooling on the step: those were its only non-reproducible kernels, deeplab_multi.py:73-79,
    95-101), and the strided 1x1 convs of layer2.0 keep the reference's stride and state_dict keys."""
    from maxsquareloss_amd.graphs.models import deeplab_multi as dm
    m = dm.DeeplabMulti(19, pretrained=False)
    hip_convs = (dm.DilatedConv3x3, dm.PointwiseConv, dm.StemConv)
    for name, mod in m.named_modules():
        if isinstance(mod, torch.nn.Conv2d) and "conv2d_list" not in name:
            assert isinstance(mod, hip_convs), name
            assert type(mod).forward is not torch.nn.Conv2d.forward, name
        assert not (isinstance(mod, torch.nn.MaxPool2d) and not isinstance(mod, dm.MaxPool)), name
    assert m.layer2[0].conv1.stride == (2, 2) and m.layer2[0].downsample[0].stride == (2, 2)
    assert m.layer2[0].stride == 2 and m.layer3[0].conv1.stride == (1, 1)
    assert isinstance(m.conv1, dm.StemConv) and isinstance(m.maxpool, dm.MaxPool)


def test_pool_output_size_matches_torch():
    from maxsquareloss_amd import ops
    for n in range(3, 70):
        for ceil in (False, True):
            ref = torch.nn.functional.max_pool2d(torch.zeros(1, 1, n, n), 3, 2, 1, ceil_mode=ceil).shape[-1]
            assert ops.pool_out(n, 3, 2, 1, ceil) == ref, (n, ceil)


def test_poly_lr_matches_reference_formula():
    from maxsquareloss_amd.tools.train_source import Trainer

    class O:
        param_groups = [{"lr": 0}, {"lr": 0}]

    class T:
        args = type("a", (), {"lr": 2.5e-4, "iter_max": 1000, "poly_power": 0.9})()
        current_iter = 100
    Trainer.poly_lr_scheduler(T, O, init_lr=2.5e-4, iter=100, max_iter=1000, power=0.9)
    assert O.param_groups[0]["lr"] == pytest.approx(2.5e-4 * 0.9 ** 0.9)
    assert O.param_groups[1]["lr"] == pytest.approx(10 * O.param_groups[0]["lr"])


# ---------------------------------------------------------------------------- DP (gloo, 2 ranks)
def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class _SinkLinear(torch.autograd.Function):
    """y = x W^T whose backward accumulates dW in place into the flat gradient buffer and returns
    None for W, as the HIP ops do (ops.grad_sink): autograd then still fires W's
    post-accumulate hook, a second report the reducer must not count."""

    @staticmethod
    def forward(ctx, x, w):
        ctx.save_for_backward(x, w)
        return x @ w.t()

    @staticmethod
    def backward(ctx, gy):
        from maxsquareloss_amd import ops
        x, w = ctx.saved_tensors
        sink = ops.grad_sink(w)
        if sink is None:
            return gy @ w, gy.t() @ x
        sink[0].add_(gy.t() @ x)
        sink[1].notify(sink[2])
        return gy @ w, None


class _SinkNet(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.l0 = torch.nn.Linear(8, 16)
        self.l1 = torch.nn.Linear(16, 16, bias=False)  # weight gradient through the sink
        self.l2 = torch.nn.Linear(16, 4)
        self.l3 = torch.nn.Linear(4, 4)  # never used: a "dead" parameter

    def forward(self, x):
        return self.l2(torch.relu(_SinkLinear.apply(torch.relu(self.l0(x)), self.l1.weight)))


def _dp_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    from maxsquareloss_amd.utils.dist import GradReducer
    from maxsquareloss_amd.utils.optim import SGD
    net = _SinkNet()
    dead = net.l3
    plist = [p for p in net.parameters()]
    opt = SGD([{"params": plist[:2] + plist[:2], "lr": 0.1}, {"params": plist[2:], "lr": 1.0}],
              lr=0.1, momentum=0.9, weight_decay=5e-4)
    red = GradReducer(opt, bucket_cap_mb=0.0002)  # ~50 floats per bucket -> several buckets
    reports = []
    opt.grads.listeners.insert(0, lambda i: reports.append(i))
    results = []
    for it in range(3):
        opt.zero_grad()
        g = torch.Generator().manual_seed(100 * it + rank)
        x1, x2 = torch.randn(5, 8, generator=g), torch.randn(3, 8, generator=g)
        net(x1).pow(2).sum().backward()      # "source" backward: local only
        red.prepare_for_backward()
        reports.clear()
        net(x2).sum().backward()             # "target" backward: overlapped reduce
        assert sorted(reports) == sorted(set(reports)), reports  # one report per parameter
        red.finish()
        results.append([p.grad.detach().numpy().copy() for p in plist] + [opt.grads.used.copy()])
        assert dead.weight.grad.abs().sum() == 0
    q.put((rank, results, red.live.copy(), opt.grad_scale))
    dist.destroy_process_group()


def test_grad_reducer_two_ranks_gloo():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_dp_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict((r, (res, live, gs)) for r, res, live, gs in (q.get(timeout=120) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # expected: the rank-sum of each rank's own (source + target) gradients
    torch.manual_seed(0)
    net = _SinkNet()
    plist = list(net.parameters())
    for it in range(3):
        total = [torch.zeros_like(p) for p in plist]
        for r in range(world):
            net.zero_grad()
            g = torch.Generator().manual_seed(100 * it + r)
            x1, x2 = torch.randn(5, 8, generator=g), torch.randn(3, 8, generator=g)
            net(x1).pow(2).sum().backward()
            net(x2).sum().backward()
            for t, p in zip(total, plist):
                if p.grad is not None:
                    t += p.grad
        for r in range(world):
            res = got[r][0][it]
            for a, b in zip(res[:-1], total):
                np.testing.assert_allclose(a, b.numpy(), rtol=1e-5, atol=1e-6)
    for r in range(world):
        assert got[r][2] == pytest.approx(1.0 / world)
        live = got[r][1]
        assert live.sum() == 5  # l0 (w, b), l1 (w, through the sink), l2 (w, b); the dead l3 excluded


def test_hot_kernels_keep_their_occupancy():
    """The compiler's resource report of the last build (Makefile: dconv.o.remarks): the forward-form
    x6 / f16x3 GEMMs and weight gradients run two workgroups (8 waves) per CU, so they must keep
    <= 256 VGPRs + AGPRs (2 waves per SIMD), and no msl kernel spills VGPRs to scratch.  (An
    epilogue change once took the forward to 242 VGPRs and one wave per SIMD: layer3 op 67 -> 90 us.)"""
    path = os.path.join(ROOT, "maxsquareloss_amd", "_lib", "obj", "dconv.o.remarks")
    if not os.path.exists(path):
        pytest.skip("no resource report: build the library first (__graft_entry__.build())")
    kern, info = None, {}
    for line in open(path):
        m = re.search(r"remark: Function Name: (\S+)", line)
        if m:
            kern = m.group(1)
            info[kern] = {}
            continue
        m = re.search(r"remark:\s+(VGPRs|AGPRs|Occupancy \[waves/SIMD\]|VGPRs Spill): (\d+)", line)
        if m and kern:
            info[kern][m.group(1)] = int(m.group(2))
    hot = [k for k in info if k.startswith("_ZN3msl14k_igemm_fwd_skILi128ELi128ELi1ELi4ELi2ELi2ELb0ELi3E")
           or k.startswith("_ZN3msl15k_igemm_fwd_sk2ILi128ELi128ELi1ELi4ELi1ELi4ELb0ELi5E")
           or k.startswith("_ZN3msl15k_igemm_fwd_sk2ILi128ELi128ELi1ELi4ELi1ELi4ELb0ELi8E")
           or k.startswith("_ZN3msl10k_wgrad_x6")]
    # the x6, f16x3 and fp16 forwards (plain, accumulating; + the plain BD and BP forms: no 3x3 call
    # accumulates) and the three weight-gradient forms
    assert len(hot) == 13, sorted(info)
    for k in hot:
        assert info[k]["Occupancy [waves/SIMD]"] >= 2, (k, info[k])
    for k, v in info.items():
        assert v.get("VGPRs Spill", 0) == 0, (k, v)


@pytest.mark.parametrize("hi,wi,ho,wo", [(65, 129, 512, 1024), (33, 65, 256, 512), (81, 161, 640, 1280),
                                         (96, 161, 760, 1280), (17, 33, 128, 256), (9, 17, 64, 128), (3, 5, 7, 300)])
def test_loss_bwd_chunk_lds_bound(hi, wi, ho, wo):
    """k_bwd_rows sizes its LDS for the widest pixel range a column chunk needs (loss.hip
    rows_wmax): check that bound against the exact ranges, with torch's fp32 source-index rounding."""
    sw = np.float32((wi - 1) / (wo - 1)) if wo > 1 else np.float32(0)
    ox = np.arange(wo, dtype=np.float32)
    i0 = np.minimum(np.floor(sw * ox).astype(np.int64), wi - 1)
    nch = max(1, min(8, wi // 32))
    per = (wi + nch - 1) // nch
    each = int(np.ceil(1.0 / float(sw))) + 2 if wi >= 2 and sw > 0 else None
    wmax = wo if each is None else min(wo, (per + 1) * each)
    for j in range(nch):
        ixa, ixb = j * per, min(wi, (j + 1) * per)
        if ixa >= ixb:
            continue
        lo = int(np.searchsorted(i0, ixa - 1, side="left"))
        hi_ = wo if ixb >= wi else int(np.searchsorted(i0, ixb, side="left"))
        assert hi_ - lo <= wmax, (j, hi_ - lo, wmax)


def _split_worker(rank, world, port, q, two_pass=False):
    """The split exchange of a captured DP step (utils/graph.py segments; solve_gta5.uda_step): bucket
    bounds end at each segment's end (set_breaks); after the first backward segment reduce_early launches
    only the buckets made of the parameters that segment finished, after the second reduce_more the next
    ones, reduce_rest the others after the last segment.  two_pass (r06, the reference's order): a source
    backward that only accumulates runs first, unarmed, inside the first segment; the exchanged buffer is
    then the rank-sum of both backwards' gradients."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    from maxsquareloss_amd.utils.dist import GradReducer
    from maxsquareloss_amd.utils.optim import SGD
    net = _SinkNet()
    plist = [p for p in net.parameters()]
    opt = SGD([{"params": plist, "lr": 0.1}], lr=0.1, momentum=0.9, weight_decay=5e-4)
    red = GradReducer(opt, bucket_cap_mb=0.0002)
    ends = [4, 5]                                 # the parameters two segments finish (backward order; the
                                                  # first two, l3, are dead)
    red.set_breaks(ends)
    g = torch.Generator().manual_seed(7 + rank)
    x = torch.randn(4, 8, generator=g)
    opt.zero_grad()
    red.prepare_for_backward()
    net(x).sum().backward()
    red.finish()                                  # first step: learns the live set
    log, real = [], red._launch
    red._launch = lambda b: (log.append(("launch", b)), real(b))[1]
    opt.zero_grad()
    red.deferred = True                           # as under a graph capture: no hooks armed
    if two_pass:
        xs = torch.randn(4, 8, generator=g)
        (2.0 * net(xs)).sum().backward()          # the source pass: accumulates, exchanges nothing
        log.append(("source", 0))
    red.prepare_for_backward()
    net(x).sum().backward()
    log.append(("segment", 1))
    red.reduce_early(ends[0])
    log.append(("segment", 2))
    red.reduce_more(ends[1])
    log.append(("segment", 3))
    red.reduce_rest()
    red.deferred = False
    q.put((rank, log, list(red.bounds), [bool(h) for h in red.has_live],
           opt.grads.flat.detach().numpy().copy(), ends))
    dist.destroy_process_group()


@pytest.mark.parametrize("two_pass", [False, True])
def test_dp_bucket_launches_interleave_gloo(two_pass):
    """Pair mode and (r06) two-pass mode: nothing launched before the first segment ends (in two-pass mode
    not during the source pass either), each bucket after the segment that finished it, every live bucket
    once, both ranks holding the same reduced buffer."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_split_worker, args=(r, world, port, q, two_pass)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict((r, rest) for r, *rest in (q.get(timeout=120) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    log, bounds, has_live, flat0, ends = got[0]
    assert all(any(hi == e for _, hi in bounds) for e in ends), (bounds, ends)  # buckets end at segment ends
    if two_pass:
        assert log[0] == ("source", 0)                    # nothing launched during the source pass
        log = log[1:]
    assert log[0] == ("segment", 1)                       # nothing launched inside the backward
    cuts = [log.index(("segment", i)) for i in (1, 2, 3)] + [len(log)]
    limits = [0] + ends + [max(hi for _, hi in bounds)]
    seen = []
    for i in range(3):
        launched = [b for k, b in log[cuts[i]:cuts[i + 1]] if k == "launch"]
        assert launched, (i, log, bounds, has_live)
        assert all(limits[i] < bounds[b][1] <= limits[i + 1] for b in launched), (i, launched, bounds)
        seen += launched
    assert seen == [b for b in range(len(bounds)) if has_live[b]]
    assert np.array_equal(flat0, got[1][3])              # both ranks hold the same reduced buffer


def test_split_segments_lead_the_flat_gradient_order():
    """The captured DP step's backward segments (model.split_cuts, r05): each segment's parameters
    follow the previous ones' in the flat buffer's backward order (UDATrainer._split_ok, so a bucket
    launched after a segment holds final gradients only), and >= 85 % of the live gradient bytes belong
    to segments before the last one (launched while the last segment replays)."""
    import types
    from maxsquareloss_amd.graphs.models.deeplab_multi import DeeplabMulti
    from maxsquareloss_amd.tools.solve_gta5 import UDATrainer
    from maxsquareloss_amd.utils.optim import SGD
    m = DeeplabMulti(19, pretrained=False)
    opt = SGD(m.optim_parameters(types.SimpleNamespace(lr=2.5e-4)), lr=2.5e-4, momentum=0.9, weight_decay=5e-4)
    assert UDATrainer._split_ok(types.SimpleNamespace(optimizer=opt, model=m))
    segs = m.split_segments()
    assert len(segs) == 1 + len(m.split_cuts)
    dead = {id(p) for n, p in m.named_parameters() if ".conv2d_list.2." in n or ".conv2d_list.3." in n}  # Q1
    live = sum(p.numel() for p in opt.grads.params if id(p) not in dead)
    early = sum(p.numel() for g in segs for p in g if id(p) not in dead)
    assert early / live >= 0.85, early / live


def _sk_tile(t, tiles_m, tiles_n, gm):
    """Host restatement of csrc/dconv_kernels.h sk_tile (r04 tile order): gm <= 1 n fastest, else
    groups of gm m-blocks with m fastest inside a group (the last group may be short)."""
    if gm <= 1:
        return t // tiles_n, t % tiles_n
    g, r = divmod(t, gm * tiles_n)
    m_in = min(gm, tiles_m - g * gm)
    tn = r // m_in
    return g * gm + (r - tn * m_in), tn


@pytest.mark.parametrize("tiles_m,tiles_n,gm", [(2, 132, 1), (8, 132, 8), (16, 132, 16), (3, 132, 3),
                                                (4, 132, 4), (5, 7, 2), (7, 3, 4), (1, 9, 1), (1, 9, 5)])
def test_sk_tile_order_is_a_bijection(tiles_m, tiles_n, gm):
    """Every stream-K tile index maps to a distinct (m-block, n-block) in range - a non-bijective order
    would leave output tiles unwritten - and with gm = tiles_m (the hybrid launches, dconv.hip
    launch_fwd_form) the m-blocks of one pixel block are consecutive tile indices."""
    seen = set()
    for t in range(tiles_m * tiles_n):
        tm, tn = _sk_tile(t, tiles_m, tiles_n, gm)
        assert 0 <= tm < tiles_m and 0 <= tn < tiles_n
        seen.add((tm, tn))
    assert len(seen) == tiles_m * tiles_n
    if gm == tiles_m:
        for t in range(tiles_m * tiles_n):
            assert _sk_tile(t, tiles_m, tiles_n, gm) == (t % tiles_m, t // tiles_m)


def test_wgrad_split_plan_query():
    """msl_conv_wgrad_split (a host-only plan query): the split (fp16-rounding in the fp16 math) weight
    gradient runs where both sides have >= 128 channels and its items fill the chip - layer3 / layer4 and
    the wide 1x1 convs at the 1024x512 pair - and the fp32-accurate tiles below 128 channels."""
    from maxsquareloss_amd import hip
    lib = hip.load(require_gpu=False)
    assert lib.msl_conv_wgrad_split(1, 9, 256, 256, 65, 129, 2) == 1    # layer3 3x3
    assert lib.msl_conv_wgrad_split(1, 9, 512, 512, 65, 129, 2) == 1    # layer4 3x3
    assert lib.msl_conv_wgrad_split(1, 1, 1024, 256, 65, 129, 2) == 1   # layer3 conv1
    assert lib.msl_conv_wgrad_split(1, 1, 256, 1024, 65, 129, 2) == 1   # layer3 conv3 (swapped operands)
    assert lib.msl_conv_wgrad_split(1, 1, 2048, 342, 65, 129, 2) == 1   # layer6 head, shift form
    assert lib.msl_conv_wgrad_split(1, 9, 64, 64, 129, 257, 2) == 0     # layer1 3x3
    assert lib.msl_conv_wgrad_split(1, 1, 64, 256, 129, 257, 2) == 0    # layer1 conv3
    assert lib.msl_conv_wgrad_split(1, 9, 64, 64, 0, 257, 2) == -3      # bad dimensions
    assert lib.msl_conv_wgrad_split(1, 3, 64, 64, 9, 9, 1) == -3        # 1 or 9 taps only
