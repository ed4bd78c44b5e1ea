"""Race screen for the HIP kernels: every op's outputs must be bit-identical run to run (fixed
summation orders), also while other kernels compete for the CUs.  Runs each op once on an idle
GPU as the reference, then N times with a background load on a second stream, and reports every
output that ever differs (count of differing elements, max |diff|)."""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from maxsquareloss_amd import ops  # noqa: E402


def make_cases(dev):
    g = torch.Generator().manual_seed(0)
    r = lambda *s, sc=1.0: (torch.randn(*s, generator=g) * sc).to(dev)  # noqa: E731
    cases = {}
    for name, (cin, cout, h, w, d) in {"l3": (256, 256, 65, 129, 2), "l4": (512, 512, 65, 129, 4),
                                       "l1": (64, 64, 129, 257, 1)}.items():
        x, wt, gy = r(1, cin, h, w), r(cout, cin, 3, 3, sc=0.05), r(1, cout, h, w)
        cache = ops.PackCache()

        def f(x=x, wt=wt, gy=gy, d=d, cache=cache):
            xg, wg = x.clone().requires_grad_(), wt.clone().requires_grad_()
            y = ops.dconv3x3(xg, wg, d, cache)
            y.backward(gy)
            return {"y": y, "dx": xg.grad, "dw": wg.grad}
        cases["dconv_" + name] = f
    for name, (cin, cout, h, w) in {"p3a": (1024, 256, 65, 129), "p3b": (256, 1024, 65, 129),
                                    "p4": (2048, 512, 65, 129)}.items():
        x, wt, gy = r(1, cin, h, w), r(cout, cin, 1, 1, sc=0.05), r(1, cout, h, w)
        cache = ops.PackCache(pointwise=True)

        def f(x=x, wt=wt, gy=gy, cache=cache):
            xg, wg = x.clone().requires_grad_(), wt.clone().requires_grad_()
            y = ops.pconv(xg, wg, cache)
            y.backward(gy)
            return {"y": y, "dx": xg.grad, "dw": wg.grad}
        cases["pconv_" + name] = f

        def f2(x=x, wt=wt, gy=gy, cache=cache):
            xg, wg = x.clone().requires_grad_(), wt.clone().requires_grad_()
            y = ops.conv1x1(xg, wg, cache)
            y.backward(gy)
            return {"y": y, "dx": xg.grad, "dw": wg.grad}
        cases["conv1x1_" + name] = f2
    for cin in (1024, 2048):
        x, gy = r(1, cin, 65, 129), r(1, 19, 65, 129)
        w0, w1, b0, b1 = r(19, cin, 3, 3, sc=0.01), r(19, cin, 3, 3, sc=0.01), r(19, sc=0.01), r(19, sc=0.01)
        cache = ops.PackCache()

        def f(x=x, gy=gy, w0=w0, w1=w1, b0=b0, b1=b1, cache=cache):
            t = [v.clone().requires_grad_() for v in (x, w0, b0, w1, b1)]
            y = ops.aspp2(t[0], t[1], t[2], t[3], t[4], 6, 12, cache)
            y.backward(gy)
            return {"y": y, **{f"g{i}": v.grad for i, v in enumerate(t)}}
        cases[f"aspp_{cin}"] = f
    for c, h, w, res in ((256, 65, 129, True), (1024, 65, 129, True), (64, 257, 513, False), (64, 129, 257, True)):
        x, rr, gy = r(1, c, h, w, sc=3.0), r(1, c, h, w), r(1, c, h, w)
        bn = torch.nn.BatchNorm2d(c).to(dev)

        def f(x=x, rr=rr, gy=gy, bn=bn, res=res):
            xg = x.clone().requires_grad_()
            rg = rr.clone().requires_grad_() if res else None
            y = ops.bn_act(bn, xg, residual=rg, relu=True)
            y.backward(gy)
            out = {"y": y, "dx": xg.grad, "dg": bn.weight.grad.clone(), "db": bn.bias.grad.clone()}
            bn.weight.grad = None
            bn.bias.grad = None
            if res:
                out["dr"] = rg.grad
            return out
        cases[f"bn_{c}_{h}"] = f
    low, low2 = r(1, 19, 65, 129, sc=4.0), r(1, 19, 65, 129, sc=4.0)
    lab = torch.randint(-1, 19, (512 * 1024,), generator=g).to(dev)

    def floss():
        out = {}
        for k, fn in (("ce", lambda t: ops.ce_up(t, lab, (512, 1024))), ("ms", lambda t: ops.maxsquare_up(t, (512, 1024))),
                      ("iw", lambda t: ops.iw_maxsquare_up(t, (512, 1024), 0.2)[0]),
                      ("mu", lambda t: ops.multi_ce_up(t, low2, (512, 1024), 0.5))):
            t = low.clone().requires_grad_()
            v = fn(t)
            v.backward()
            out[k] = v.detach().reshape(1)
            out[k + "_d"] = t.grad
        t = low.clone().requires_grad_()
        up = ops.upsample_bilinear(t, (512, 1024))
        up.backward(torch.ones_like(up))
        out["up"], out["up_d"] = up, t.grad
        return out
    cases["losses"] = floss
    return cases


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=12)
    ap.add_argument("--only", default="")
    ap.add_argument("--form", default="bf16x6")
    a = ap.parse_args()
    dev = torch.device("cuda")
    ops.set_f32_form(a.form)
    cases = make_cases(dev)
    noise_src = torch.randn(64 << 20, device=dev)
    noise_dst = torch.empty_like(noise_src)
    side = torch.cuda.Stream()
    bad = 0
    for name, fn in cases.items():
        if a.only and a.only not in name:
            continue
        ref = {k: v.detach().clone() for k, v in fn().items()}
        torch.cuda.synchronize()
        diffs = {}
        for rep in range(a.reps):
            if rep % 2 == 1:  # odd repetitions: compete with a memory-bound kernel stream
                with torch.cuda.stream(side):
                    for _ in range(4):
                        noise_dst.copy_(noise_src)
                        noise_src.mul_(1.0000001)
            out = fn()
            torch.cuda.synchronize()
            for k, v in out.items():
                d = (v.detach() != ref[k]) & ~(torch.isnan(v.detach()) & torch.isnan(ref[k]))
                n = int(d.sum())
                if n:
                    md = (v.detach() - ref[k]).abs().max().item()
                    c, m = diffs.get(k, (0, 0.0))
                    diffs[k] = (c + 1, max(m, md))
        status = "OK " if not diffs else "RACE"
        bad += bool(diffs)
        print(f"{status} {name:16s} {diffs if diffs else ''}", flush=True)
    print(f"{bad} op(s) not bit-reproducible", flush=True)


if __name__ == "__main__":
    main()
