"""Golden-vector generator - ORACLE tooling, runs only in the survey container.

Imports the reference's own graphs/models/deeplab_multi.py and utils/loss.py by
file path (the package __init__s pull in torchvision/tensorboardX, which are
absent; the two files themselves only need torch) and records their outputs on
seeded inputs into tests/golden/*.npz.  The reference sources never leave this
container; only these input/output vectors are committed.

    python oracle/gen_golden.py [--ref /root/reference] [--out tests/golden]

Fixtures:
  loss_kat.npz   MaxSquare / IW-MaxSquare / CE(ignore=-1) / multi-level label on seeded
                 logits for C in {19, 16, 13}, plus an argmax-tie case and an all-ignored
                 CE case (nan, quirk Q8): values, histograms, weights, d loss / d logits.
  conv_kat.npz   dilated 3x3 convs (d=2 @256ch, d=4 @512ch) and both ASPP heads
                 (reference Classifier_Module incl. its early return, Q1) at 17x33:
                 outputs and gradients as fp64 per-channel sums + sampled elements.
  sgd_kat.npz    torch.optim.SGD(foreach=False) over duplicated lists (k = 1, 3, 4) and
                 a grad=None parameter, 3 steps (quirk Q2).
  optim_lists.json  the reference's optim_parameters() group lists by name.
  step_cfg1.npz  reference model (counter init, seed 12345) at 512x256: UDA iterations
                 (maxsquare multi=False, IW_maxsquare multi=True) and train_source
                 iterations: loss scalars, logits summaries, grad / param checksums,
                 BN running-stat sums.
"""
import argparse
import importlib.util
import json
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from maxsquareloss_amd.utils.synthetic import counter_normal, init_weights, synthetic_image, synthetic_labels  # noqa: E402


def load_ref(ref_root):
    def load(name, path):
        spec = importlib.util.spec_from_file_location(name, path)
        m = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(m)
        return m
    dm = load("ref_deeplab_multi", os.path.join(ref_root, "graphs/models/deeplab_multi.py"))
    ls = load("ref_loss", os.path.join(ref_root, "utils/loss.py"))
    return dm, ls


def sample_idx(n, k=64, seed=0):
    return np.unique(np.linspace(0, n - 1, k).astype(np.int64))


def summ(t, prefix, out):
    """fp64 per-channel sums, global sum/abs-sum, and sampled elements of a (1,C,...) or (C,...) tensor."""
    a = t.detach().double().cpu().numpy()
    c = a.reshape(a.shape[0] if a.ndim != 4 or a.shape[0] != 1 else a.shape[1], -1)
    out[prefix + "_chsum"] = c.sum(1)
    out[prefix + "_sum"] = np.array(a.sum())
    out[prefix + "_abssum"] = np.array(np.abs(a).sum())
    flat = a.reshape(-1)
    idx = sample_idx(flat.size)
    out[prefix + "_idx"] = idx
    out[prefix + "_sample"] = flat[idx].astype(np.float32)


def gen_loss_kat(ls, out_dir):
    out = {}
    for C in (19, 16, 13):
        low = torch.from_numpy(counter_normal(77, f"loss_low_{C}", C * 9 * 17, 4.0)).view(1, C, 9, 17)
        low2 = torch.from_numpy(counter_normal(78, f"loss_low2_{C}", C * 9 * 17, 4.0)).view(1, C, 9, 17)
        y = synthetic_labels(64, 128, C, 900 + C)
        out[f"C{C}_low"] = low.numpy()
        out[f"C{C}_low2"] = low2.numpy()
        out[f"C{C}_y"] = y.numpy()
        hw = (64, 128)
        # MaxSquare (loss.py:104-119) on softmax of the upsampled logits
        lr = low.clone().requires_grad_()
        pred = F.interpolate(lr, size=hw, mode="bilinear", align_corners=True)
        P = F.softmax(pred, dim=1)
        l_ms = ls.MaxSquareloss(num_class=C)(pred, P)
        l_ms.backward()
        out[f"C{C}_ms"] = np.array(l_ms.item(), np.float32)
        out[f"C{C}_ms_dlow"] = lr.grad.numpy()
        # IW MaxSquare (loss.py:69-102)
        lr = low.clone().requires_grad_()
        pred = F.interpolate(lr, size=hw, mode="bilinear", align_corners=True)
        P = F.softmax(pred, dim=1)
        iw = ls.IW_MaxSquareloss(num_class=C, ratio=0.2)
        l_iw = iw(pred, P)
        l_iw.backward()
        _, arg = torch.max(P.detach(), 1)
        hist = torch.histc(arg.float(), bins=C + 1, min=-1, max=C - 1)[1:]
        out[f"C{C}_iw"] = np.array(l_iw.item(), np.float32)
        out[f"C{C}_iw_hist"] = hist.numpy().astype(np.int64)
        out[f"C{C}_iw_dlow"] = lr.grad.numpy()
        out[f"C{C}_argmax"] = arg.numpy().astype(np.int8)
        # CE(ignore=-1)
        lr = low.clone().requires_grad_()
        pred = F.interpolate(lr, size=hw, mode="bilinear", align_corners=True)
        l_ce = torch.nn.CrossEntropyLoss(ignore_index=-1)(pred, y)
        l_ce.backward()
        out[f"C{C}_ce"] = np.array(l_ce.item(), np.float32)
        out[f"C{C}_ce_dlow"] = lr.grad.numpy()
        # multi-level guidance (solve_gta5.py:206-213), threshold 0.95 and 0.5
        for thr in (0.95, 0.5):
            lr = low.clone().requires_grad_()
            pred_2 = F.interpolate(lr, size=hw, mode="bilinear", align_corners=True)
            pred = F.interpolate(low2, size=hw, mode="bilinear", align_corners=True)
            P, P2 = F.softmax(pred, dim=1), F.softmax(pred_2, dim=1)
            maxpred, _ = torch.max(P.detach(), dim=1)
            maxpred_2, _ = torch.max(P2.detach(), dim=1)
            pc = (P + P2) / 2
            _, argc = torch.max(pc, dim=1)
            mask = (maxpred > thr) | (maxpred_2 > thr)
            label_2 = torch.where(mask, argc, torch.ones(1, dtype=torch.long) * -1)
            l_m = torch.nn.CrossEntropyLoss(ignore_index=-1)(pred_2, label_2)
            l_m.backward()
            t = str(thr).replace(".", "p")
            out[f"C{C}_multi{t}_label"] = label_2.numpy().astype(np.int8)
            out[f"C{C}_multi{t}_ce"] = np.array(l_m.item(), np.float32)
            out[f"C{C}_multi{t}_dlow"] = lr.grad.numpy()
    # argmax ties: equal logits across classes -> first index (torch.max on CPU)
    tie = torch.zeros(1, 19, 4, 8)
    tie[:, 3] = 1.0
    tie[:, 7] = 1.0
    tie[0, :, 0, 0] = 0.0
    P = F.softmax(tie, 1)
    iw = ls.IW_MaxSquareloss(num_class=19, ratio=0.2)
    out["tie_logits"] = tie.numpy()
    out["tie_iw"] = np.array(iw(tie, P).item(), np.float32)
    _, arg = torch.max(P, 1)
    out["tie_argmax"] = arg.numpy().astype(np.int8)
    # all-ignored CE -> nan (Q8)
    l = torch.nn.CrossEntropyLoss(ignore_index=-1)(torch.zeros(1, 19, 4, 8), torch.full((1, 4, 8), -1))
    out["allignored_ce"] = np.array(l.item(), np.float32)
    np.savez_compressed(os.path.join(out_dir, "loss_kat.npz"), **out)


def gen_conv_kat(dm, out_dir):
    out = {}
    h, w = 17, 33
    torch.manual_seed(0)
    for name, planes, dil in (("d2", 256, 2), ("d4", 512, 4)):
        blk = dm.Bottleneck(planes * 4, planes, dilation=dil)
        conv = blk.conv2  # the reference's dilated conv module (deeplab_multi.py:17-18)
        with torch.no_grad():
            conv.weight.copy_(torch.from_numpy(counter_normal(5, f"conv_{name}_w", conv.weight.numel(), 0.01)).view_as(conv.weight))
        x = torch.from_numpy(counter_normal(6, f"conv_{name}_x", planes * h * w)).view(1, planes, h, w).requires_grad_()
        gy = torch.from_numpy(counter_normal(7, f"conv_{name}_gy", planes * h * w)).view(1, planes, h, w)
        y = conv(x)
        y.backward(gy)
        summ(y, f"{name}_y", out)
        summ(x.grad, f"{name}_dx", out)
        summ(conv.weight.grad, f"{name}_dw", out)
        out[f"{name}_meta"] = np.array([planes, h, w, dil])
    for head, cin in (("aspp5", 1024), ("aspp6", 2048)):
        mod = dm.Classifier_Module(cin, [6, 12, 18, 24], [6, 12, 18, 24], 19)
        with torch.no_grad():
            for i, c in enumerate(mod.conv2d_list):
                c.weight.copy_(torch.from_numpy(counter_normal(8, f"{head}_w{i}", c.weight.numel(), 0.01)).view_as(c.weight))
                c.bias.copy_(torch.from_numpy(counter_normal(9, f"{head}_b{i}", 19, 0.01)))
        x = torch.from_numpy(counter_normal(10, f"{head}_x", cin * h * w)).view(1, cin, h, w).requires_grad_()
        gy = torch.from_numpy(counter_normal(11, f"{head}_gy", 19 * h * w)).view(1, 19, h, w)
        y = mod(x)
        y.backward(gy)
        summ(y, f"{head}_y", out)
        summ(x.grad, f"{head}_dx", out)
        for i in range(4):
            c = mod.conv2d_list[i]
            out[f"{head}_w{i}_hasgrad"] = np.array(c.weight.grad is not None)
            if c.weight.grad is not None:
                summ(c.weight.grad, f"{head}_dw{i}", out)
                out[f"{head}_db{i}"] = c.bias.grad.numpy()
    np.savez_compressed(os.path.join(out_dir, "conv_kat.npz"), **out)


def gen_sgd_kat(out_dir):
    shapes = [(8, 3, 3, 3), (16,), (4, 8, 3, 3), (5,), (7,)]
    mult = [1, 3, 4, 1, 3]
    out = {"shapes": np.array([int(np.prod(s)) for s in shapes]), "mult": np.array(mult)}
    params = []
    for i, s in enumerate(shapes):
        v = torch.from_numpy(counter_normal(20, f"sgd_p{i}", int(np.prod(s)))).view(s)
        out[f"p{i}_init"] = v.numpy()
        params.append(v.clone().requires_grad_())
    g0 = [p for p, k in zip(params[:4], mult[:4]) for _ in range(k)]
    # param 4 is duplicated but never gets a gradient (skipped, like dead ASPP branches)
    g0 += [params[4]] * mult[4]
    opt = torch.optim.SGD([{"params": g0[:-3] + g0[-3:], "lr": 0.01}], lr=0.01, momentum=0.9,
                          weight_decay=5e-4, foreach=False)
    for step in range(3):
        for i, p in enumerate(params[:4]):
            g = torch.from_numpy(counter_normal(21 + step, f"sgd_g{i}", p.numel())).view(p.shape)
            out[f"g{i}_step{step}"] = g.numpy()
            p.grad = g.clone()
        params[4].grad = None
        opt.step()
        for i, p in enumerate(params):
            out[f"p{i}_step{step}"] = p.detach().numpy().copy()
    np.savez_compressed(os.path.join(out_dir, "sgd_kat.npz"), **out)


def ref_model(dm, num_classes=19, seed=12345):
    m = dm.DeeplabMulti(num_classes=num_classes, pretrained=False)
    init_weights(m, seed)
    return m


def gen_optim_lists(dm, out_dir):
    m = ref_model(dm)
    names = {id(p): n for n, p in m.named_parameters()}

    class A:
        lr = 2.5e-4
    groups = m.optim_parameters(A)
    lists = [[names[id(p)] for p in g["params"]] for g in groups]
    with open(os.path.join(out_dir, "optim_lists.json"), "w") as f:
        json.dump({"group0": lists[0], "group1": lists[1]}, f)


def gen_step(dm, ls, out_dir, h=256, w=512):
    out = {}
    cfgs = {
        "ms": dict(target_mode="maxsquare", multi=False, lambda_target=0.1),
        "iwmulti": dict(target_mode="IW_maxsquare", multi=True, lambda_target=0.09),
    }
    common = dict(lr=2.5e-4, iter_max=200000, lambda_seg=0.1, IW_ratio=0.2, threshold=0.95)
    torch.set_num_threads(os.cpu_count())
    names = None
    for tag, cfg in cfgs.items():
        cfg = {**common, **cfg}
        m = ref_model(dm)
        m.train()
        names = [n for n, _ in m.named_parameters()]

        class A:
            lr = cfg["lr"]
        opt = torch.optim.SGD(m.optim_parameters(A), lr=cfg["lr"], momentum=0.9, weight_decay=5e-4, foreach=False)
        ce = torch.nn.CrossEntropyLoss(ignore_index=-1)
        tl = (ls.MaxSquareloss(num_class=19) if cfg["target_mode"] == "maxsquare"
              else ls.IW_MaxSquareloss(num_class=19, ratio=0.2))
        for it in range(2):
            # solve_gta5.py:336-383 restated around the reference's model + loss modules
            lr = cfg["lr"] * (1 - float(it) / cfg["iter_max"]) ** 0.9
            opt.param_groups[0]["lr"], opt.param_groups[1]["lr"] = lr, 10 * lr
            xs, ys = synthetic_image(h, w, it), synthetic_labels(h, w, 19, it)
            xt = synthetic_image(h, w, 500 + it)
            pred, pred_2 = m(xs)
            if it == 0:
                summ(pred, f"{tag}_it0_src_x2", out)
                summ(pred_2, f"{tag}_it0_src_x1", out)
            loss = ce(pred, ys)
            loss_ = loss
            if cfg["multi"]:
                loss_2 = cfg["lambda_seg"] * ce(pred_2, ys)
                loss_ = loss_ + loss_2
                out[f"{tag}_it{it}_loss_seg_2"] = np.array(loss_2.item())
            loss_.backward()
            out[f"{tag}_it{it}_loss_seg"] = np.array(loss.item())
            pred, pred_2 = m(xt)
            if it == 0:
                summ(pred, f"{tag}_it0_tgt_x2", out)
            P = F.softmax(pred, dim=1)
            P2 = F.softmax(pred_2, dim=1)
            lt = cfg["lambda_target"] * tl(pred, P)
            total = lt
            if cfg["target_mode"] == "IW_maxsquare":
                _, arg = torch.max(P.detach(), 1)
                out[f"{tag}_it{it}_hist"] = torch.histc(arg.float(), bins=20, min=-1, max=18)[1:].numpy().astype(np.int64)
            if cfg["multi"]:
                maxpred, _ = torch.max(P.detach(), dim=1)
                maxpred_2, _ = torch.max(P2.detach(), dim=1)
                _, argc = torch.max((P + P2) / 2, dim=1)
                mask = (maxpred > cfg["threshold"]) | (maxpred_2 > cfg["threshold"])
                label_2 = torch.where(mask, argc, torch.ones(1, dtype=torch.long) * -1)
                lt2 = cfg["lambda_seg"] * cfg["lambda_target"] * ce(pred_2, label_2)
                total = total + lt2
                out[f"{tag}_it{it}_loss_target_2"] = np.array(lt2.item())
                out[f"{tag}_it{it}_nvalid2"] = np.array(int((label_2 >= 0).sum()))
            total.backward()
            out[f"{tag}_it{it}_loss_target"] = np.array(lt.item())
            if it == 0:
                out[f"{tag}_it0_gradsum"] = np.array([0.0 if p.grad is None else p.grad.double().sum().item() for p in m.parameters()])
                out[f"{tag}_it0_gradabs"] = np.array([0.0 if p.grad is None else p.grad.double().abs().sum().item() for p in m.parameters()])
                out[f"{tag}_it0_hasgrad"] = np.array([p.grad is not None for p in m.parameters()])
            opt.step()
            opt.zero_grad()
        out[f"{tag}_param_sum"] = np.array([p.double().sum().item() for p in m.parameters()])
        out[f"{tag}_param_abssum"] = np.array([p.double().abs().sum().item() for p in m.parameters()])
        out[f"{tag}_bn_mean_sum"] = np.array([b.double().sum().item() for n, b in m.named_buffers() if n.endswith("running_mean")])
        out[f"{tag}_bn_var_sum"] = np.array([b.double().sum().item() for n, b in m.named_buffers() if n.endswith("running_var")])
        print(tag, {k: float(v) for k, v in out.items() if k.startswith(tag) and "loss" in k}, flush=True)
    # config 1: tools/train_source.py, 2 iterations (multi=True default)
    m = ref_model(dm)
    m.train()

    class A:
        lr = 2.5e-4
    opt = torch.optim.SGD(m.optim_parameters(A), lr=2.5e-4, momentum=0.9, weight_decay=5e-4, foreach=False)
    ce = torch.nn.CrossEntropyLoss(ignore_index=-1)
    for it in range(2):
        lr = 2.5e-4 * (1 - float(it) / 200000) ** 0.9
        opt.param_groups[0]["lr"], opt.param_groups[1]["lr"] = lr, 10 * lr
        x, y = synthetic_image(h, w, 100 + it), synthetic_labels(h, w, 19, 100 + it)
        pred, pred_2 = m(x)
        cur = ce(pred, y) + 0.1 * ce(pred_2, y)
        opt.zero_grad()
        cur.backward()
        opt.step()
        out[f"src_it{it}_loss"] = np.array(cur.item())
    out["src_param_sum"] = np.array([p.double().sum().item() for p in m.parameters()])
    out["param_names"] = np.array(names)
    out["hw"] = np.array([h, w])
    np.savez_compressed(os.path.join(out_dir, "step_cfg1.npz"), **out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--out", default=os.path.join(os.path.dirname(HERE), "tests", "golden"))
    ap.add_argument("--skip-step", action="store_true")
    a = ap.parse_args()
    if not os.path.isdir(a.ref):
        print("reference not present; goldens are committed, nothing to do")
        return
    os.makedirs(a.out, exist_ok=True)
    dm, ls = load_ref(a.ref)
    gen_loss_kat(ls, a.out)
    gen_conv_kat(dm, a.out)
    gen_sgd_kat(a.out)
    gen_optim_lists(dm, a.out)
    if not a.skip_step:
        gen_step(dm, ls, a.out)


if __name__ == "__main__":
    main()
