"""Where does iteration 0 of two identical UDA trainers diverge (tests/test_gpu_graph.py's setup)?

Three trainers from the same counter-generated init run iteration 0 of the test's UDA step on the same
inputs: A eagerly on the default stream, B on a side stream (as GraphedStep._first does), C on the
default stream after the caching allocator's free blocks were filled with NaN (a kernel that reads
memory it did not write shows up there).  Every module output of the source and target forwards is
recorded by hooks and compared in forward order; the first differing module is printed per pair."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from maxsquareloss_amd.tools.solve_gta5 import UDATrainer, build_parser  # noqa: E402
from maxsquareloss_amd.tools.train_source import init_args  # noqa: E402
from maxsquareloss_amd.utils.synthetic import synthetic_image, synthetic_labels  # noqa: E402

H, W = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (256, 512)


def trainer():
    argv = ["--crop_size", f"{W},{H}", "--target_crop_size", f"{W},{H}", "--imagenet_pretrained", "False",
            "--save_dir", "", "--target_mode", "IW_maxsquare", "--multi", "True", "--lambda_target", "0.09",
            "--iter_max", "1000", "--graph", "False"]
    args, _, _ = init_args(build_parser().parse_args(argv))
    tr = UDATrainer(args, cuda=True)
    tr.optimizer.zero_grad()
    return tr


def run(tr, stream=None):
    outs = []
    hs = [m.register_forward_hook(lambda mod, i, o, n=n: outs.append(
        (n, (o[0] if isinstance(o, tuple) else o).detach().clone()))) for n, m in tr.model.named_modules() if n]
    xs = synthetic_image(H, W, 40).cuda()
    ys = synthetic_labels(H, W, 19, 40).cuda()
    xt = synthetic_image(H, W, 540).cuda()
    if stream is None:
        tr.uda_step(xs, ys, xt)
    else:
        stream.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(stream):
            tr.uda_step(xs, ys, xt)
        torch.cuda.current_stream().wait_stream(stream)
    torch.cuda.synchronize()
    for h in hs:
        h.remove()
    scal = {k: getattr(tr, k).item() for k in ("loss_val", "loss_target", "loss_target_2")}
    grads = [p.grad.detach().clone() if p.grad is not None else None for p in tr.model.parameters()]
    params = [p.detach().clone() for p in tr.model.parameters()]
    return outs, scal, params


def compare(tag, a, b):
    oa, sa, pa = a
    ob, sb, pb = b
    print(f"== {tag}: scalars {sa} vs {sb}", flush=True)
    nd = 0
    for (na, x), (nb, y) in zip(oa, ob):
        if x.shape != y.shape or not torch.equal(x, y):
            d = ((x - y).abs().max() / x.abs().max().clamp_min(1e-30)).item() if x.shape == y.shape else -1
            print(f"   differs #{len(oa) and [n for n, _ in oa].index(na)} {na} {tuple(x.shape)} rel {d:.3e} "
                  f"nan {torch.isnan(y).any().item()}", flush=True)
            nd += 1
            if nd >= 8:
                break
    npd = sum(int(not torch.equal(x, y)) for x, y in zip(pa, pb))
    print(f"   modules compared {len(oa)}, differing shown {nd}; params differing after the step: {npd}", flush=True)


warm = trainer()
warm.uda_step(synthetic_image(H, W, 39).cuda(), synthetic_labels(H, W, 19, 39).cuda(), synthetic_image(H, W, 539).cuda())
torch.cuda.synchronize()
del warm
ra = run(trainer())
rb = run(trainer(), torch.cuda.Stream())
# fill the allocator's free blocks with NaN, then run C
torch.cuda.synchronize()
junk = []
free, _ = torch.cuda.mem_get_info()
cached = torch.cuda.memory_reserved() - torch.cuda.memory_allocated()
print("reserved-but-free bytes", cached, flush=True)
for sz in (1 << 30, 1 << 28, 1 << 26, 1 << 24, 1 << 22, 1 << 20, 1 << 16):
    try:
        while torch.cuda.memory_reserved() - torch.cuda.memory_allocated() >= sz and len(junk) < 4000:
            junk.append(torch.full((sz // 4,), float("nan"), device="cuda"))
    except RuntimeError:
        pass
del junk
torch.cuda.synchronize()
rc = run(trainer())
rd = run(trainer())
compare("A default vs B side stream", ra, rb)
compare("A vs C (NaN-filled free blocks)", ra, rc)
compare("A vs D (default again)", ra, rd)
