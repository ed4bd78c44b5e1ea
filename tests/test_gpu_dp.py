"""The real data-parallel path, two ranks on the one leased GPU (GPU only).

Both ranks run the real DeeplabMulti (256x128) through UDATrainer with the
GradReducer of utils/dist.py on a gloo process group (RCCL refuses two ranks on
one device; the reducer code is backend-agnostic).  The HIP ops report their
weight gradients through ops.grad_sink -> FlatGrads.notify, not AccumulateGrad
hooks, so this is the test of that path's bucket countdown:
  - iteration A learns the live set (the first finish() reduces everything);
  - iteration B runs armed: every live bucket must be launched by the countdown
    during the target backward (before finish()), only after every live
    parameter of the bucket has reported its final gradient, in bucket order;
    the reduced flat buffer must equal the sum over ranks of each bucket's
    local contents at its launch (stream-ordered snapshots), exactly.
Every kernel of the step is deterministic (no library kernel since r03), so the
exchange is checked exactly: each bucket against the launch-time snapshots of both
ranks' local gradients.
"""
import gc
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

H, W = 128, 256


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _grads(tr, xs, ys, xt):
    """The gradient part of UDATrainer.uda_step (solve_gta5.py:344-381), no optimizer step."""
    tr.optimizer.zero_grad()
    tr.train_source(tr.model(xs), ys)
    tr.train_target(tr.model(xt))
    if tr.reducer:
        tr.reducer.finish()
    torch.cuda.synchronize()
    return tr.optimizer.grads.flat.detach().cpu().clone()


def _worker(rank, world, port, q, outdir):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                          WORLD_SIZE=str(world), LOCAL_RANK="0")
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from maxsquareloss_amd.tools.solve_gta5 import UDATrainer, build_parser
        from maxsquareloss_amd.tools.train_source import init_args
        from maxsquareloss_amd.utils.synthetic import synthetic_image, synthetic_labels
        argv = ["--crop_size", f"{W},{H}", "--target_crop_size", f"{W},{H}", "--imagenet_pretrained", "False",
                "--save_dir", "", "--target_mode", "IW_maxsquare", "--multi", "True", "--lambda_target", "0.09"]
        args, _, _ = init_args(build_parser().parse_args(argv))
        tr = UDATrainer(args, cuda=True)
        red = tr.reducer
        assert red is not None and red.world == world
        seed = 1000 * rank + 7
        xs = synthetic_image(H, W, seed).cuda()
        ys = synthetic_labels(H, W, 19, seed).cuda()
        xt = synthetic_image(H, W, 500 + seed).cuda()
        _grads(tr, xs, ys, xt)                    # A: learns the live set
        events = []                               # ("notify", param) / ("launch", bucket, snapshot)
        flat = tr.optimizer.grads
        orig_launch, orig_finish = red._launch, red.finish
        in_finish = [False]

        def on_grad(i):
            events.append(("notify", i))

        def launch(b):
            from maxsquareloss_amd import ops
            ops.wgrad_join()  # the bucket's weight gradients may still be on the side stream
            a, e = red._elem_range(b)
            events.append(("launch", b, flat.flat[a:e].clone(), in_finish[0]))  # stream-ordered copy
            if os.environ.get("MSL_DP_SYNC_LAUNCH"):
                torch.cuda.synchronize()  # diagnostic: hand gloo a settled buffer
            orig_launch(b)

        def finish():
            in_finish[0] = True
            orig_finish()
            in_finish[0] = False
        orig_prepare = red.prepare_for_backward

        def prepare():
            events.append(("arm", -1))
            orig_prepare()
        flat.listeners.insert(0, on_grad)
        red._launch, red.finish, red.prepare_for_backward = launch, finish, prepare
        reduced = _grads(tr, xs, ys, xt)          # B: armed, overlapped exchange
        flat.listeners.remove(on_grad)
        armed_at = next(k for k, ev in enumerate(events) if ev[0] == "arm")
        events = events[armed_at + 1:]  # the target backward (the source backward is not armed)
        log = [(ev[0], ev[1], ev[3]) if ev[0] == "launch" else ev for ev in events]
        snaps = {ev[1]: ev[2].cpu().numpy() for ev in events if ev[0] == "launch"}
        np.save(os.path.join(outdir, f"reduced{rank}.npy"), reduced.numpy())
        np.savez(os.path.join(outdir, f"snaps{rank}.npz"), **{str(b): v for b, v in snaps.items()})
        names = [n for n, p in tr.model.named_parameters() if p.requires_grad][::-1]
        q.put((rank, "ok", log, red.has_live, red.live.copy(), list(red.bounds), tr.optimizer.grad_scale,
               [red._elem_range(b) for b in range(len(red.bounds))], list(flat.offsets), names))
        dist.destroy_process_group()
    except Exception as e:  # surface the failure to the parent instead of hanging it
        import traceback
        q.put((rank, "error", traceback.format_exc() + repr(e)))
        raise


def test_grad_reducer_real_model_two_ranks(tmp_path):
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, str(tmp_path))) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    try:
        for _ in range(world):
            item = q.get(timeout=240)
            assert item[1] == "ok", item[2]
            got[item[0]] = item[2:]
        for p in procs:
            p.join(timeout=60)
            assert p.exitcode == 0
    finally:
        for p in procs:  # never leave a rank behind (it would hold the GPU and the test runner)
            if p.is_alive():
                p.kill()
                p.join(timeout=10)
    snaps = [np.load(os.path.join(tmp_path, f"snaps{r}.npz")) for r in range(world)]
    for r in range(world):
        reduced = np.load(os.path.join(tmp_path, f"reduced{r}.npy"))
        log, has_live, live, bounds, gscale, ranges, offs, names = got[r]
        assert gscale == pytest.approx(1.0 / world)
        assert len(bounds) > 3 and live.sum() > 300
        launches = [e for e in log if e[0] == "launch"]
        # every bucket with a live parameter launched exactly once, in order, by the countdown
        # during the target backward (not by finish())
        assert [e[1] for e in launches] == [b for b in range(len(bounds)) if has_live[b]], launches
        assert not any(e[2] for e in launches), launches
        # every live parameter reports exactly once in the armed backward
        from collections import Counter
        cnt = Counter(e[1] for e in log if e[0] == "notify")
        assert all(cnt[i] == 1 for i in range(len(live)) if live[i]), \
            [(names[i], cnt[i]) for i in range(len(live)) if live[i] and cnt[i] != 1][:10]
        # ... and only after every live parameter of the bucket had reported its gradient
        seen = set()
        for e in log:
            if e[0] == "notify":
                seen.add(e[1])
            else:
                lo, hi = bounds[e[1]]
                missing = [i for i in range(lo, hi) if live[i] and i not in seen]
                assert not missing, (e[1], missing)
        # the reduced buffer = the rank-sum of what each rank held when the bucket launched
        for b in range(len(bounds)):
            if not has_live[b]:
                continue
            a, e = ranges[b]
            want = snaps[0][str(b)].astype(np.float64) + snaps[1][str(b)].astype(np.float64)
            got_b = reduced[a:e].astype(np.float64)
            want = want.astype(np.float32).astype(np.float64)
            if not np.array_equal(got_b, want):
                lo, hi = bounds[b]
                detail = [(names[i], float(np.abs(got_b[offs[i] - a:offs[i + 1] - a] - want[offs[i] - a:offs[i + 1] - a]).max()),
                           float(np.abs(want[offs[i] - a:offs[i + 1] - a]).max())) for i in range(lo, hi)]
                other = np.load(os.path.join(tmp_path, f"reduced{1 - r}.npy"))[a:e].astype(np.float64)
                i = next(i for i in range(lo, hi) if detail[i - lo][1] > 0)
                sl = slice(offs[i] - a, offs[i + 1] - a)
                d = got_b[sl] - want[sl]
                s0, s1 = snaps[0][str(b)][sl].astype(np.float64), snaps[1][str(b)][sl].astype(np.float64)
                k = int(np.abs(d).argmax())
                raise AssertionError((r, b, [x for x in detail if x[1] > 0], "ranks agree:",
                                      bool(np.array_equal(got_b[sl], other[sl])), "n differing", int((d != 0).sum()),
                                      "of", d.size, "at argmax: got", got_b[sl][k], "s0", s0[k], "s1", s1[k],
                                      "other rank", other[sl][k]))


def _graph_worker(rank, world, port, q, pair=True):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                          WORLD_SIZE=str(world), LOCAL_RANK="0")
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from maxsquareloss_amd.tools.solve_gta5 import UDATrainer, build_parser
        from maxsquareloss_amd.tools.train_source import init_args
        from maxsquareloss_amd.utils.synthetic import synthetic_image, synthetic_labels
        out = {}
        for graph in (False, True):
            argv = ["--crop_size", f"{W},{H}", "--target_crop_size", f"{W},{H}", "--imagenet_pretrained", "False",
                    "--save_dir", "", "--target_mode", "IW_maxsquare", "--multi", "True", "--lambda_target", "0.09",
                    "--iter_max", "1000", "--graph", str(graph), "--pair", str(pair)]
            args, _, _ = init_args(build_parser().parse_args(argv))
            tr = UDATrainer(args, cuda=True)
            tr.optimizer.zero_grad()
            losses = []
            log = []
            for it in range(4):
                if graph and it == 3:  # the host's order of segment replays and bucket launches
                    gs, red = tr._graphed, tr.reducer
                    for i, g in enumerate(gs.graphs):
                        g.replay = (lambda f, i: lambda: (log.append(("replay", i)), f())[1])(g.replay, i)
                    red._launch = (lambda f: lambda b: (log.append(("launch", b)), f(b))[1])(red._launch)
                seed = 1000 * rank + it
                tr.uda_step(synthetic_image(H, W, seed).cuda(), synthetic_labels(H, W, 19, seed).cuda(),
                            synthetic_image(H, W, 500 + seed).cuda())
                torch.cuda.synchronize()
                losses.append((tr.loss_val.item(), tr.loss_target.item(), tr.loss_target_2.item()))
            if graph:
                assert tr._graphed is not None and tr._graphed.replays == 3 and tr._graphed.graph_update is not None
                # the backward replays as segments split at layer3's output and inside layer3 (split_cuts);
                # after each segment the buckets it finished launch (bucket bounds end at every segment's
                # end), the rest after the last one
                ends = list(np.cumsum([len(g) for g in tr.model.split_segments()]))
                assert len(tr._graphed.graphs) == 1 + len(ends), len(tr._graphed.graphs)
                assert all(any(hi == e for _, hi in red.bounds) for e in ends), (ends, red.bounds)
                assert log[0] == ("replay", 0), log
                seen = []
                for i in range(len(ends) + 1):
                    r0 = log.index(("replay", i))
                    r1 = log.index(("replay", i + 1)) if i < len(ends) else len(log)
                    got_b = [b for k, b in log[r0:r1] if k == "launch"]
                    lo = ends[i - 1] if i else 0
                    hi = ends[i] if i < len(ends) else len(red.flat.params)
                    assert got_b and all(lo < red.bounds[b][1] <= hi for b in got_b), (i, got_b, lo, hi)
                    seen += got_b
                assert seen == [b for b in range(len(red.bounds)) if red.has_live[b]], log
            out[graph] = (losses, torch.cat([p.detach().reshape(-1) for p in tr.model.parameters()]).cpu().numpy())
            del tr
        q.put((rank, "ok", out))
        dist.destroy_process_group()
    except Exception as e:  # surface the failure to the parent instead of hanging it
        import traceback
        q.put((rank, "error", traceback.format_exc() + repr(e)))
        raise


@pytest.mark.parametrize("pair", [True, False])
def test_graphed_dp_step_matches_eager_dp(pair):
    """The captured data-parallel step (utils/graph.py: the forward/backward passes as graphs split at
    layer3's output and inside layer3, the exchange of each segment's gradients launched after its
    replay, the rest of the exchange after the last, then the graph of the SGD step) against the eager DP
    step with the overlapped bucket countdown, 2 ranks (gloo) x 4 UDA iterations: every loss and
    every parameter bit-identical (the step has no library kernel and the 2-rank sum is exact in
    either order), and the two replicas' parameters identical after every run (one exchange per
    iteration keeps data-parallel replicas in lock step).  r06: also in two-pass mode (--pair False, the
    reference's source-then-target order), whose captured step now cuts the target backward the same way."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_graph_worker, args=(r, world, port, q, pair)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    try:
        for _ in range(world):
            item = q.get(timeout=300)
            assert item[1] == "ok", item[2]
            got[item[0]] = item[2]
        for p in procs:
            p.join(timeout=60)
            assert p.exitcode == 0
    finally:
        for p in procs:
            if p.is_alive():
                p.kill()
                p.join(timeout=10)
    for r in range(world):
        (le, pe), (lg, pg) = got[r][False], got[r][True]
        assert le == lg, (r, le, lg)
        assert np.array_equal(pe, pg), (r, int((pe != pg).sum()))
    for graph in (False, True):
        assert np.array_equal(got[0][graph][1], got[1][graph][1]), graph


def _rccl_worker(port, q):
    """One rank on the GPU with an RCCL ("nccl") process group and the exchange forced on (--dp_exchange)
    against the same run without a process group: the captured, segmented DP step on the real collective
    library (the all-reduce at one rank is the identity)."""
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1",
                          LOCAL_RANK="0")
        import torch.distributed as dist
        from maxsquareloss_amd.tools.solve_gta5 import UDATrainer, build_parser
        from maxsquareloss_amd.tools.train_source import init_args
        from maxsquareloss_amd.utils.synthetic import synthetic_image, synthetic_labels
        out, log = {}, []

        def mark(m):
            print(f"[rccl worker] {m}", file=sys.stderr, flush=True)

        for dp in (False, True):
            mark(f"trainer dp={dp}")
            argv = ["--crop_size", f"{W},{H}", "--target_crop_size", f"{W},{H}", "--imagenet_pretrained", "False",
                    "--save_dir", "", "--target_mode", "IW_maxsquare", "--multi", "True", "--lambda_target", "0.09",
                    "--iter_max", "1000", "--graph", "True", "--dp_exchange", str(dp)]
            args, _, _ = init_args(build_parser().parse_args(argv))
            tr = UDATrainer(args, cuda=True)
            mark("trainer built")
            assert (tr.reducer is not None) == dp and dist.is_initialized() == dp
            if dp:
                assert dist.get_backend() == "nccl" and tr.reducer.always
            losses = []
            for it in range(4):
                if dp and it == 3:
                    red = tr.reducer
                    red._launch = (lambda f: lambda b: (log.append(b), f(b))[1])(red._launch)
                    works = []
                    import torch.distributed as d2
                    orig = d2.all_reduce
                    d2.all_reduce = lambda *a, **k: works.append(1) or orig(*a, **k)
                tr.uda_step(synthetic_image(H, W, it).cuda(), synthetic_labels(H, W, 19, it).cuda(),
                            synthetic_image(H, W, 500 + it).cuda())
                torch.cuda.synchronize()
                mark(f"iteration {it} done")
                if dp and it == 3:
                    d2.all_reduce = orig
                    assert len(works) == len(log) > 0, (len(works), log)
                losses.append((tr.loss_val.item(), tr.loss_target.item(), tr.loss_target_2.item()))
            if dp:
                assert tr._graphed is not None and len(tr._graphed.graphs) == 1 + len(tr.model.split_segments())
                assert log == [b for b in range(len(tr.reducer.bounds)) if tr.reducer.has_live[b]], log
            out[dp] = (losses, torch.cat([p.detach().reshape(-1) for p in tr.model.parameters()]).cpu().numpy())
            del tr
            gc.collect()
        dist.destroy_process_group()
        q.put(("ok", out))
    except Exception as e:
        import traceback
        q.put(("error", traceback.format_exc() + repr(e)))
        raise


def test_rccl_world1_graphed_dp_matches_single_gpu():
    """RCCL on the hardware (r05): the segmented, graph-captured DP step with a real "nccl" (RCCL)
    process group at one rank (--dp_exchange: every live bucket all-reduced between the segment replays,
    counted) gives the same losses and parameters bit for bit as the single-GPU step without a process
    group, over 4 UDA iterations.  (Two ranks need two GPUs for RCCL; the 2-rank exchange itself is
    tested on gloo above.)"""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(_free_port(), q))
    p.start()
    try:
        import queue
        import time
        deadline = time.time() + 300
        while True:  # a worker that dies (an abort in the runtime) fails the test instead of hanging it
            try:
                status, got = q.get(timeout=5)
                break
            except queue.Empty:
                assert p.is_alive(), f"RCCL worker died, exit code {p.exitcode}"
                assert time.time() < deadline, "RCCL worker timed out"
        assert status == "ok", got
        p.join(timeout=60)
        assert p.exitcode == 0
    finally:
        if p.is_alive():
            p.kill()
            p.join(timeout=10)
    (l0, p0), (l1, p1) = got[False], got[True]
    assert l0 == l1, (l0, l1)
    assert np.array_equal(p0, p1), int((p0 != p1).sum())


def _cfg2_worker(rank, world, port, q, outdir):
    """One eager UDA iteration of BASELINE configs[2] (IW-MaxSquare, 1024x512, multi False, lambda_t 0.1)
    on one of two data-parallel replicas; the initial weights (rank 0), the losses, the IW histogram
    and the parameters after the step go to files."""
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                          WORLD_SIZE=str(world), LOCAL_RANK="0")
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from maxsquareloss_amd.tools.solve_gta5 import UDATrainer, build_parser
        from maxsquareloss_amd.tools.train_source import init_args
        from maxsquareloss_amd.utils.synthetic import synthetic_image, synthetic_labels
        h, w = CFG2_HW
        argv = ["--crop_size", f"{w},{h}", "--target_crop_size", f"{w},{h}", "--imagenet_pretrained", "False",
                "--save_dir", "", "--target_mode", "IW_maxsquare", "--multi", "False", "--lambda_target", "0.1",
                "--iter_max", "200000"]
        args, _, _ = init_args(build_parser().parse_args(argv))
        tr = UDATrainer(args, cuda=True)
        assert tr.reducer is not None and tr.reducer.world == world and tr.pair
        if rank == 0:
            torch.save({k: v.detach().cpu() for k, v in tr.model.state_dict().items()},
                       os.path.join(outdir, "init.pt"))
        seed = 300 + rank
        xs, ys, xt = synthetic_image(h, w, seed), synthetic_labels(h, w, 19, seed), synthetic_image(h, w, 600 + seed)
        tr.optimizer.zero_grad()
        tr.uda_step(xs.cuda(), ys.cuda(), xt.cuda())
        torch.cuda.synchronize()
        np.savez(os.path.join(outdir, f"params{rank}.npz"),
                 **{n: p.detach().cpu().numpy() for n, p in tr.model.named_parameters()})
        q.put((rank, "ok", tr.loss_val.item(), tr.loss_target.item(),
               tr.target_loss.last_hist.cpu().numpy().astype(np.int64)))
        dist.destroy_process_group()
    except Exception as e:  # surface the failure to the parent instead of hanging it
        import traceback
        q.put((rank, "error", traceback.format_exc() + repr(e)))
        raise


CFG2_HW = (512, 1024)


def test_dp_cfg2_full_size_matches_oracle(tmp_path):
    """BASELINE configs[2] at its real size as a data-parallel step: two replicas (gloo, one GPU) each
    run the pair-mode UDA iteration on their own 1024x512 images and exchange gradients once.  Held
    against the CPU oracle of the same data-parallel step (each replica's gradients from its images,
    averaged, one SGD step - oracle.uda_grads): every replica's losses within 1e-3 of the oracle at its
    images, its IW histogram within 0.1 % of the pixels, both replicas' parameters identical after the
    step, and the update per tensor within 3x the fp32 oracle's own distance to an fp64 oracle (the
    bars of test_gpu_configs.py)."""
    from oracle import msl_oracle as orc
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_cfg2_worker, args=(r, world, port, q, str(tmp_path))) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    try:
        for _ in range(world):
            item = q.get(timeout=600)
            assert item[1] == "ok", item[2]
            got[item[0]] = item[2:]
        for p in procs:
            p.join(timeout=120)
            assert p.exitcode == 0
    finally:
        for p in procs:
            if p.is_alive():
                p.kill()
                p.join(timeout=10)
    h, w = CFG2_HW
    sd0 = torch.load(os.path.join(str(tmp_path), "init.pt"), weights_only=True)
    cfg = dict(lr=2.5e-4, iter_max=200000, lambda_seg=0.1, IW_ratio=0.2, threshold=0.95, target_mode="IW_maxsquare",
               multi=False, lambda_target=0.1)
    from maxsquareloss_amd.tools.solve_gta5 import build_parser
    from maxsquareloss_amd.tools.train_source import init_args
    args, _, _ = init_args(build_parser().parse_args(["--imagenet_pretrained", "False", "--save_dir", ""]))
    cfg.update(lr=args.lr, lambda_seg=args.lambda_seg, IW_ratio=args.IW_ratio, threshold=args.threshold)
    res = {}
    for dtype in (torch.float32, torch.float64):
        model = orc.Model(sd0, 19, dtype=dtype)
        opt = orc.SGDMult(model.params, model.names, cfg["lr"])
        lr = orc.poly_lr(cfg["lr"], 0, cfg["iter_max"])
        opt.groups[0]["lr"], opt.groups[1]["lr"] = lr, 10 * lr
        outs = []
        for r in range(world):
            seed = 300 + r
            outs.append(orc.uda_grads(model, orc_img(seed, h, w), orc_lab(seed, h, w), orc_img(600 + seed, h, w), cfg))
        with torch.no_grad():
            for p in model.params.values():
                if p.grad is not None:
                    p.grad.mul_(1.0 / world)  # the replicas' mean (the SGD kernel's grad_scale)
        opt.step()
        res[dtype] = (model, outs)
    (m32, outs32), (m64, _) = res[torch.float32], res[torch.float64]
    for r in range(world):
        loss_s, loss_t, hist = got[r]
        o = outs32[r]
        for k, v in (("loss_seg", loss_s), ("loss_target", loss_t)):
            rel = abs(v - o[k]) / max(abs(o[k]), 1e-30)
            print(f"cfg2 dp rank {r} {k}: gpu {v:.7g} oracle {o[k]:.7g} rel {rel:.2e}")
            assert v == pytest.approx(o[k], rel=1e-3), (r, k, v, o[k])
        flips = int(np.abs(hist - o["hist"]).sum()) // 2
        print(f"cfg2 dp rank {r} IW histogram: {flips} argmax flips of {h * w} pixels")
        assert hist.sum() == o["hist"].sum() == h * w and flips <= 0.001 * h * w
    p0, p1 = np.load(os.path.join(str(tmp_path), "params0.npz")), np.load(os.path.join(str(tmp_path), "params1.npz"))
    e_gpu_all = e_cpu_all = 0.0
    for n in m32.names:
        assert np.array_equal(p0[n], p1[n]), n  # one exchange keeps the replicas in lock step
        init = sd0[n].double()
        du = torch.from_numpy(p0[n]).double() - init
        dr = m32.params[n].detach().double() - init
        d64 = m64.params[n].detach() - init
        if d64.abs().max() == 0:
            assert du.abs().max() == 0, n  # dead parameters (Q1) untouched
            continue
        e_gpu, e_cpu = (du - d64).norm().item(), (dr - d64).norm().item()
        e_gpu_all += e_gpu ** 2
        e_cpu_all += e_cpu ** 2
        assert e_gpu <= max(3 * e_cpu, 1e-3 * d64.norm().item()), (n, e_gpu, e_cpu)
    print(f"cfg2 dp SGD update vs fp64: gpu {e_gpu_all ** 0.5:.3e} cpu-fp32 {e_cpu_all ** 0.5:.3e}")
    assert e_gpu_all <= 4 * e_cpu_all


def orc_img(seed, h, w):
    from maxsquareloss_amd.utils.synthetic import synthetic_image
    return synthetic_image(h, w, seed)


def orc_lab(seed, h, w):
    from maxsquareloss_amd.utils.synthetic import synthetic_labels
    return synthetic_labels(h, w, 19, seed)
