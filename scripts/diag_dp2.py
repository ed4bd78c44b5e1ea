"""Diagnostic: does arming the reducer change the local gradient?  (C = armed + gloo, D = armed + no-op
collective, E = local again after C and D)."""
import os, sys, socket
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np, torch, torch.multiprocessing as mp

H, W = 128, 256

def grads(tr, xs, ys, xt):
    tr.optimizer.zero_grad()
    tr.train_source(tr.model(xs), ys)
    tr.train_target(tr.model(xt))
    if tr.reducer:
        tr.reducer.finish()
    torch.cuda.synchronize()
    return tr.optimizer.grads.flat.detach().cpu().double().numpy().copy()

def worker(rank, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE="2", LOCAL_RANK="0")
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=2)
    from maxsquareloss_amd.tools.solve_gta5 import UDATrainer, build_parser
    from maxsquareloss_amd.tools.train_source import init_args
    from maxsquareloss_amd.utils.synthetic import synthetic_image, synthetic_labels
    import maxsquareloss_amd.utils.dist as ud
    argv = ["--crop_size", f"{W},{H}", "--target_crop_size", f"{W},{H}", "--imagenet_pretrained", "False",
            "--save_dir", "", "--target_mode", sys.argv[1], "--multi", sys.argv[2], "--lambda_target", "0.09"]
    args, _, _ = init_args(build_parser().parse_args(argv))
    tr = UDATrainer(args, cuda=True)
    red = tr.reducer
    seed = 1000 * rank + 7
    xs, ys, xt = synthetic_image(H, W, seed).cuda(), synthetic_labels(H, W, 19, seed).cuda(), synthetic_image(H, W, 500 + seed).cuda()
    grads(tr, xs, ys, xt)
    tr.reducer = None
    B1 = grads(tr, xs, ys, xt)
    tr.reducer = red
    C = grads(tr, xs, ys, xt)
    class Done:
        def wait(self): pass
    real = ud.dist.all_reduce
    ud.dist.all_reduce = lambda t, group=None, async_op=False: Done()
    D = grads(tr, xs, ys, xt)
    ud.dist.all_reduce = real
    tr.reducer = None
    E = grads(tr, xs, ys, xt)
    offs = tr.optimizer.grads.offsets
    names = [n for n, p in tr.model.named_parameters() if p.requires_grad][::-1]
    def rel(a, b):
        out = []
        for i in range(len(offs) - 1):
            lo, hi = int(offs[i]), int(offs[i + 1])
            out.append(np.abs(a[lo:hi] - b[lo:hi]).max() / max(np.abs(b[lo:hi]).max(), 1e-30))
        return np.array(out)
    np.save(f"/tmp/B1_{rank}.npy", B1)
    q.put((rank, rel(D, B1), rel(E, B1), names, list(offs)))
    q.put((rank, "C", C))
    dist.destroy_process_group()

if __name__ == "__main__":
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]
    ctx = mp.get_context("spawn"); q = ctx.Queue()
    procs = [ctx.Process(target=worker, args=(r, port, q)) for r in range(2)]
    [p.start() for p in procs]
    res, Cs = {}, {}
    try:
        for _ in range(4):
            it = q.get(timeout=300)
            if isinstance(it[1], str):
                Cs[it[0]] = it[2]
            else:
                res[it[0]] = it[1:]
        [p.join(60) for p in procs]
    finally:
        for p in procs:
            if p.is_alive():
                p.kill()
    exp = np.load("/tmp/B1_0.npy") + np.load("/tmp/B1_1.npy")
    for r in range(2):
        dB, eB, names, offs = res[r]
        C = Cs[r]
        cr = []
        for i in range(len(offs) - 1):
            lo, hi = int(offs[i]), int(offs[i + 1])
            cr.append(np.abs(C[lo:hi] - exp[lo:hi]).max() / max(np.abs(exp[lo:hi]).max(), 1e-30))
        cr = np.array(cr)
        print(f"rank {r}: armed+noop vs local max {dB.max():.3e} (param {names[dB.argmax()]}); local after vs before max {eB.max():.3e}; "
              f"armed+gloo vs sum max {cr.max():.3e} (param {names[cr.argmax()]}), #params > 1e-5: {(cr > 1e-5).sum()}")
