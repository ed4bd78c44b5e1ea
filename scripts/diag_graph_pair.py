"""Where does the first replay of the captured UDA step diverge from the eager step (tests/test_gpu_graph.py's
setup)?  Forward hooks registered before iteration 0 clone every module output; in the graphed trainer the
clones made while capturing are rewritten by every replay, so after the first replay they hold iteration 1's
values.  Prints the first differing modules of iteration 1 (eager vs replay).  argv: pair True|False."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from maxsquareloss_amd.tools.solve_gta5 import UDATrainer, build_parser  # noqa: E402
from maxsquareloss_amd.tools.train_source import init_args  # noqa: E402
from maxsquareloss_amd.utils.synthetic import synthetic_image, synthetic_labels  # noqa: E402

H, W = 256, 512
PAIR = sys.argv[1] if len(sys.argv) > 1 else "True"
FORM = sys.argv[2] if len(sys.argv) > 2 else None
THIRD = os.environ.get("DIAG_THIRD", "1") == "1"


def trainer(graph, pair=None):
    argv = ["--crop_size", f"{W},{H}", "--target_crop_size", f"{W},{H}", "--imagenet_pretrained", "False",
            "--save_dir", "", "--target_mode", "IW_maxsquare", "--multi", "True", "--lambda_target", "0.09",
            "--iter_max", "1000", "--graph", str(graph), "--pair", pair or PAIR] + (["--f32_form", FORM] if FORM else [])
    args, _, _ = init_args(build_parser().parse_args(argv))
    tr = UDATrainer(args, cuda=True)
    tr.optimizer.zero_grad()
    return tr


def inputs(it):
    return (synthetic_image(H, W, 40 + it).cuda(), synthetic_labels(H, W, 19, 40 + it).cuda(),
            synthetic_image(H, W, 540 + it).cuda())


def hook(tr, rec):
    def f(mod, i, o, n):
        t = o[0] if isinstance(o, tuple) else o
        rec.setdefault(n, []).append(t.detach().clone())
    return [m.register_forward_hook(lambda mod, i, o, n=n: f(mod, i, o, n)) for n, m in tr.model.named_modules() if n]


E, G = trainer(False), trainer(True)
T = trainer(False, "False") if THIRD else E
snaps = {}
for tag, tr in (("E", E), ("G", G), ("T", T)):
    buf = torch.zeros_like(tr.optimizer.grads.flat)
    snaps[tag] = buf
    step = tr.optimizer.step

    def wrapped(closure=None, _step=step, _buf=buf, _tr=tr):
        _buf.copy_(_tr.optimizer.grads.flat)  # the gradient the step reads (captured in G's graph)
        return _step(closure)
    tr.optimizer.step = wrapped
re, rg = {}, {}
he, hg = hook(E, re), hook(G, rg)
# every (pointer, count) of absmax partials handed to a conv entry point, cloned at the call (captured in
# G's graph, so after the replay G's list holds iteration 1's values); per trainer, by the current owner
from maxsquareloss_amd import ops as _ops  # noqa: E402
_pp0 = _ops._pp
PARTS = {"cur": None}


def _pp_rec(q):
    lst = PARTS.get(PARTS["cur"])
    if lst is not None and q is not None:
        import traceback
        where = " < ".join(f"{f.name}:{f.lineno}" for f in traceback.extract_stack()[-4:-1])
        lst.append((where, q[0].detach().clone()))
    return _pp0(q)


_ops._pp = _pp_rec
for it in range(2):
    for tag, tr in (("E", E), ("G", G), ("T", T)) if THIRD else (("E", E), ("G", G)):
        PARTS["cur"] = tag
        if it == 0:
            PARTS[tag] = []
        tr.uda_step(*inputs(it))
        PARTS["cur"] = None
    torch.cuda.synchronize()
    print(f"it {it}: E loss {E.loss_val.item():.9g} {E.loss_target.item():.9g}  G loss {G.loss_val.item():.9g} "
          f"{G.loss_target.item():.9g}", flush=True)
# E: records [it0, it1] per module call; G: [it0 eager, capture clones (= it1 after the replay)]
names = list(re.keys())
nd = 0
for n in names:
    a, b = re[n], rg.get(n, [])
    if len(a) != len(b):
        print("count mismatch", n, len(a), len(b))
        continue
    half = len(a) // 2
    for k in range(len(a)):
        x, y = a[k], b[k]
        if not torch.equal(x, y):
            d = ((x - y).abs().max() / x.abs().max().clamp_min(1e-30)).item()
            print(f"differs: {n} call {k} ({'it0' if k < half else 'it1'}) {tuple(x.shape)} rel {d:.3e} "
                  f"nan {torch.isnan(y).any().item()}", flush=True)
            nd += 1
    if nd >= 12:
        break
print("modules", len(names), "differences shown", nd)
# the parameters after iteration 0's update (eager in both) and the packs
pd = [n for (n, p), q in zip(E.model.named_parameters(), G.model.parameters()) if not torch.equal(p, q)]
print("params differing after it1:", len(pd), pd[:6])

offs = E.optimizer.grads.offsets
pn = {id(p): n for n, p in E.model.named_parameters()}
order = [pn.get(id(p), "?") for p in E.optimizer.grads.params]
ge, gg = snaps["E"].cpu(), snaps["G"].cpu()
bad = [(order[i], float((ge[offs[i]:offs[i + 1]] - gg[offs[i]:offs[i + 1]]).abs().max()),
        float(ge[offs[i]:offs[i + 1]].abs().max())) for i in range(len(order))
       if not torch.equal(ge[offs[i]:offs[i + 1]], gg[offs[i]:offs[i + 1]])]
print("it1 gradients differing (name, max diff, max):", len(bad), bad[:8])
mb = []
for (n, p), q in zip(E.model.named_parameters(), G.model.parameters()):
    a, b = E.optimizer.state.get(p, {}).get("momentum_buffer"), G.optimizer.state.get(q, {}).get("momentum_buffer")
    if a is not None and b is not None and not torch.equal(a, b):
        mb.append((n, float((a - b).abs().max())))
print("momentum differing:", len(mb), mb[:6])
gt = snaps["T"].cpu()
for i in range(len(order)):
    if order[i] == "layer2.0.downsample.0.weight":
        sl = slice(int(offs[i]), int(offs[i + 1]))
        for tag, v in (("E", ge[sl]), ("G", gg[sl])):
            print(f"{tag} vs two-pass T: max diff {float((v - gt[sl]).abs().max()):.3e} of {float(gt[sl].abs().max()):.3e}; "
                  f"ratio stats {(v / gt[sl]).median().item():.4g}")
pe, pg = PARTS["E"], PARTS["G"]
print("partials calls E", len(pe), "G(capture)", len(pg))
pe, pg = pe[len(pe) // 2:], pg[len(pg) // 2:]
for k, ((a0, a), (b0, b)) in enumerate(zip(pe, pg)):
    if a.shape != b.shape or not torch.equal(a, b):
        print(f"  partials call {k} differ: n {a.numel()} E max {float(a.max()):.3e} min {float(a.min()):.3e} | "
              f"G max {float(b.max()):.3e} min {float(b.min()):.3e} | {a0}")
