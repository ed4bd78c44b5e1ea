"""Diagnostic for tests/test_gpu_dp.py: which parameters differ between local and reduced gradients."""
import os, sys, socket
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch, torch.multiprocessing as mp
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import test_gpu_dp as T

def main():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]
    out = "/tmp/diagdp"; os.makedirs(out, exist_ok=True)
    ctx = mp.get_context("spawn"); q = ctx.Queue()
    procs = [ctx.Process(target=T._worker, args=(r, 2, port, q, out)) for r in range(2)]
    [p.start() for p in procs]
    got = {}
    for _ in range(2):
        it = q.get(timeout=240); got[it[0]] = it[2:]
    [p.join(60) for p in procs]
    local = [np.load(f"{out}/local{r}.npy") for r in range(2)]
    exp = local[0].astype(np.float64) + local[1]
    from maxsquareloss_amd.graphs.models.deeplab_multi import DeeplabMulti
    m = DeeplabMulti(19, False)
    names = [n for n, p in m.named_parameters() if p.requires_grad][::-1]
    for r in range(2):
        red = np.load(f"{out}/reduced{r}.npy")
        log, has_live, live, bounds, gs, offs = got[r]
        print("rank", r, "bounds", bounds[:4], "launch log", log)
        for i in range(len(offs) - 1):
            lo, hi = int(offs[i]), int(offs[i + 1])
            e = exp[lo:hi]; a = red[lo:hi]
            d = np.abs(a - e).max(); sc = max(np.abs(e).max(), 1e-30)
            if d > 1e-5 * sc:
                l0 = np.abs(local[0][lo:hi]).max()
                print(f"  {i:3d} {names[i]:34s} bucket {[b for b,(x,y) in enumerate(bounds) if x<=i<y]} rel {d/sc:.3e} "
                      f"| red-l0 {np.abs(a-local[0][lo:hi]).max()/sc:.3e} red-l1 {np.abs(a-local[1][lo:hi]).max()/sc:.3e}")
if __name__ == "__main__":
    main()
