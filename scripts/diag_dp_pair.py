"""Diagnostic: the eager data-parallel step with the overlapped bucket countdown vs the same step with
the exchange deferred to after the backward (what the captured DP step does), in pair and two-pass
mode, 2 ranks (gloo) on one GPU.  Prints per-parameter differences of the exchanged gradient."""
import os, sys, socket
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np, torch, torch.multiprocessing as mp

H, W = 128, 256


def worker(rank, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE="2", LOCAL_RANK="0")
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=2)
    from maxsquareloss_amd.tools.solve_gta5 import UDATrainer, build_parser
    from maxsquareloss_amd.tools.train_source import init_args
    from maxsquareloss_amd.utils.synthetic import synthetic_image, synthetic_labels
    out = {}
    for pair in ("True", "False"):
        for mode in ("overlap", "deferred", "local"):
            argv = ["--crop_size", f"{W},{H}", "--target_crop_size", f"{W},{H}", "--imagenet_pretrained", "False",
                    "--save_dir", "", "--target_mode", "IW_maxsquare", "--multi", "True", "--lambda_target", "0.09",
                    "--iter_max", "1000", "--pair", pair]
            args, _, _ = init_args(build_parser().parse_args(argv))
            tr = UDATrainer(args, cuda=True)
            tr.optimizer.zero_grad()
            red = tr.reducer
            res = []
            for it in range(3):
                seed = 1000 * rank + it
                xs, ys, xt = (synthetic_image(H, W, seed).cuda(), synthetic_labels(H, W, 19, seed).cuda(),
                              synthetic_image(H, W, 500 + seed).cuda())
                tr.poly_lr_scheduler(optimizer=tr.optimizer, init_lr=tr.args.lr)
                if it == 0 or mode == "overlap":
                    tr._uda_grads(xs, ys, xt)
                    red.finish()
                elif mode == "deferred":
                    red.deferred = True
                    tr._uda_grads(xs, ys, xt)
                    red.deferred = False
                    red.reduce_all()
                else:  # local gradient only, then the deferred exchange
                    red.deferred = True
                    tr._uda_grads(xs, ys, xt)
                    red.deferred = False
                    torch.cuda.synchronize()
                    loc = tr.optimizer.grads.flat.detach().cpu().numpy().copy()
                    red.reduce_all()
                    out[(pair, "localgrad", it)] = loc
                torch.cuda.synchronize()
                g = tr.optimizer.grads.flat.detach().cpu().numpy().copy()
                res.append((tr.loss_val.item(), tr.loss_target.item()))
                out[(pair, mode, it)] = g
                tr._uda_update()
                tr.current_iter += 1
            out[(pair, mode, "loss")] = res
            names = [n for n, p in tr.model.named_parameters() if p.requires_grad][::-1]
            out["offs"] = np.asarray(tr.optimizer.grads.offsets)
            out["names"] = [n for n in (getattr(p, "_msl_name", None) for p in tr.optimizer.grads.params)]
            out["pnames"] = {id(p): n for n, p in tr.model.named_parameters()}
            out["order"] = [out["pnames"].get(id(p), "?") for p in tr.optimizer.grads.params]
            del tr, red
    q.put((rank, out))
    dist.destroy_process_group()


def main():
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=600) for _ in range(2))
    for p in ps:
        p.join(timeout=60)
    for r in range(2):
        o = got[r]
        offs, order = o["offs"], o["order"]
        for pair in ("True", "False"):
            print(f"rank {r} pair {pair} losses: overlap {o[(pair, 'overlap', 'loss')]}")
            print(f"rank {r} pair {pair} losses: deferred {o[(pair, 'deferred', 'loss')]}")
            for it in range(3):
                a, b, c = o[(pair, "overlap", it)], o[(pair, "deferred", it)], o[(pair, "local", it)]
                diff = [(order[i], float(np.abs(a[offs[i]:offs[i + 1]] - b[offs[i]:offs[i + 1]]).max()))
                        for i in range(len(order)) if not np.array_equal(a[offs[i]:offs[i + 1]], b[offs[i]:offs[i + 1]])]
                print(f"  it {it}: overlap vs deferred: {len(diff)} params differ {diff[:8]}; deferred vs local-run "
                      f"equal: {np.array_equal(b, c)}")
    for pair in ("True", "False"):
        for it in range(1, 3):
            la, lb = got[0][(pair, "localgrad", it)], got[1][(pair, "localgrad", it)]
            ex = (la.astype(np.float64) + lb).astype(np.float32)
            for mode in ("overlap", "deferred"):
                g = got[0][(pair, mode, it)] if it == 1 else None
                if g is not None:
                    offs, order = got[0]["offs"], got[0]["order"]
                    bad = [order[i] for i in range(len(order)) if not np.array_equal(g[offs[i]:offs[i + 1]], ex[offs[i]:offs[i + 1]])]
                    print(f"pair {pair} it {it} {mode}: exchanged != local sum for {len(bad)} params {bad[:8]}")


if __name__ == "__main__":
    main()
