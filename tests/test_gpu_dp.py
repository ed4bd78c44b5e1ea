"""The real data-parallel path, two ranks on the one leased GPU (GPU only).

Both ranks run the real DeeplabMulti (256x128) through UDATrainer with the
GradReducer of utils/dist.py on a gloo process group (RCCL refuses two ranks on
one device; the reducer code is backend-agnostic).  The HIP ops report their
weight gradients through ops.grad_sink -> FlatGrads.notify, not AccumulateGrad
hooks, so this is the test of that path's bucket countdown:
  - iteration A learns the live set (the first finish() reduces everything);
  - iteration B computes each rank's local gradient with the reducer detached;
  - iteration C runs armed: every live bucket must be launched by the countdown
    during the target backward (before finish()), and the reduced flat buffer
    must equal the sum of the two ranks' local gradients.
No optimizer step runs between A, B and C, so the three see the same weights.
"""
import os
import socket

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
        tr.reducer = None
        local = _grads(tr, xs, ys, xt)            # B: this rank's own gradient ...
        again = _grads(tr, xs, ys, xt)            # ... twice: the run-to-run noise of the step
        tr.reducer = red
        log = []
        in_finish = [False]
        orig_launch, orig_finish = red._launch, red.finish

        def launch(b):
            log.append((b, in_finish[0]))
            orig_launch(b)

        def finish():
            in_finish[0] = True
            orig_finish()
            in_finish[0] = False
        red._launch, red.finish = launch, finish
        reduced = _grads(tr, xs, ys, xt)          # C: armed, overlapped exchange
        # the gradient buffers go through files: 2 x 174 MB do not belong in a pipe
        np.save(os.path.join(outdir, f"local{rank}.npy"), local.numpy())
        np.save(os.path.join(outdir, f"again{rank}.npy"), again.numpy())
        np.save(os.path.join(outdir, f"reduced{rank}.npy"), reduced.numpy())
        q.put((rank, "ok", log, red.has_live, red.live.copy(), list(red.bounds), tr.optimizer.grad_scale,
               tr.optimizer.grads.offsets.copy()))
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
    local = [np.load(os.path.join(tmp_path, f"local{r}.npy")) for r in range(world)]
    again = [np.load(os.path.join(tmp_path, f"again{r}.npy")) for r in range(world)]
    expect = local[0].astype(np.float64) + local[1].astype(np.float64)
    for r in range(world):
        reduced = np.load(os.path.join(tmp_path, f"reduced{r}.npy"))
        log, has_live, live, bounds, gscale, offs = got[r]
        assert gscale == pytest.approx(1.0 / world)
        # every bucket with a live parameter was launched exactly once, by the countdown during the
        # target backward (before finish()), in bucket order
        launched = [b for b, _ in log]
        assert launched == [b for b in range(len(bounds)) if has_live[b]], launched
        assert not any(late for _, late in log), log
        assert len(bounds) > 3 and live.sum() > 300
        # the reduced buffer = rank-sum of the local gradients.  The local gradient itself is not
        # bit-reproducible run to run (MIOpen's stem / stride-2 convs; amplified through the bs=1
        # network and the thresholded pseudo-label of the multi-level guidance CE), so the bar per
        # parameter is 1e-5 of its scale plus 4x the measured run-to-run change of the two ranks.
        assert np.abs(expect).max() > 0
        for i in range(len(offs) - 1):
            lo, hi = int(offs[i]), int(offs[i + 1])
            e = expect[lo:hi]
            a = reduced[lo:hi].astype(np.float64)
            noise = sum(np.abs(again[k][lo:hi].astype(np.float64) - local[k][lo:hi]).max() for k in range(world))
            tol = 1e-5 * max(np.abs(e).max(), 1e-30) + 4 * noise
            assert np.abs(a - e).max() <= tol, (i, np.abs(a - e).max(), np.abs(e).max(), noise)
