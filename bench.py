"""bench.py - training images/s of the MI355X DeepLabv2/ResNet-101 MaxSquare UDA step.

    python bench.py --gpus N --steps K --warmup W          (N > 1: launched by torchrun)

A "step" is one iteration of tools/solve_gta5.py:335-387: one source image
(fwd, CE, bwd) + one target image (fwd, MaxSquare, bwd) + the gradient
all-reduce (N > 1) + the SGD step, i.e. 2 images per rank per step (by default
the two images run as one pair: per-image BN statistics, one GEMM per conv).  Workload =
BASELINE.json configs[1]: GTA5->Cityscapes MaxSquare, 1024x512, bs=1/GPU,
random-init (counter generator) weights, synthetic inputs already in HBM,
--multi False, lambda_target 0.1, fp32.  Scaling is weak (bs=1 per GPU).

Printed (rank 0, one JSON line): value = total images/s over all ranks, the
roofline of the dominant kernel (layer3's dilated 3x3 forward, timed live with
HIP events on its stream during the timed steps), the CPU baseline (the oracle's
PyTorch-CPU restatement of the same step, a bounded sample on this host), and
the relative loss delta of the first iteration vs that CPU reference.
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from maxsquareloss_amd import ops  # noqa: E402
from maxsquareloss_amd.tools.solve_gta5 import UDATrainer, build_parser  # noqa: E402
from maxsquareloss_amd.tools.train_source import init_args  # noqa: E402
from maxsquareloss_amd.utils.synthetic import synthetic_image, synthetic_labels  # noqa: E402

METRIC = json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X dense FP32 matrix peak (MI355X_MICROARCH.md)
BF16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X dense BF16 matrix peak (no sparsity)
HBM_PEAK_GBS = 8000.0


def feat_hw(n):
    """Spatial size of layer3/4 for an input side n: stem 7x7/2, maxpool 3/2 ceil_mode, layer2 1x1/2."""
    n = (n - 1) // 2 + 1
    m = -(-(n + 2 - 3) // 2) + 1
    if (m - 1) * 2 >= n + 1:
        m -= 1
    return (m - 1) // 2 + 1


def pool_out(n, k, s, p, ceil):
    """torch's pooling output size (dilation 1)."""
    num = n + 2 * p - (k - 1) - 1 + ((s - 1) if ceil else 0)
    o = num // s + 1
    if ceil and (o - 1) * s >= n + p:
        o -= 1
    return o


def conv_gflop(H, W, C):
    """(forward GFLOP of every conv of DeeplabMulti for one H x W image, the stem's share): 2*cin*cout*k*k
    per output pixel over the stem, the 33 Bottlenecks (3 / 4 / 23 / 3) with their downsamples and both
    live ASPP branches of both heads (deeplab_multi.py:8-48, 51-66, 69-101).  1024x512, C = 19:
    741.44 and 2.47."""
    hs, ws = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    hm, wm = pool_out(hs, 3, 2, 1, True), pool_out(ws, 3, 2, 1, True)
    h2, w2 = (hm - 1) // 2 + 1, (wm - 1) // 2 + 1
    stem = 2.0 * 64 * 3 * 49 * hs * ws
    f, inpl = stem, 64
    for planes, blocks, p in ((64, 3, hm * wm), (128, 4, h2 * w2), (256, 23, h2 * w2), (512, 3, h2 * w2)):
        for b in range(blocks):
            f += 2.0 * inpl * planes * p + 2.0 * planes * planes * 9 * p + 2.0 * planes * planes * 4 * p
            if b == 0:
                f += 2.0 * inpl * planes * 4 * p  # downsample
            inpl = planes * 4
    f += 2 * (2.0 * 1024 * C * 9 * h2 * w2) + 2 * (2.0 * 2048 * C * 9 * h2 * w2)
    return f / 1e9, stem / 1e9


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--height", type=int, default=512)
    ap.add_argument("--width", type=int, default=1024)
    ap.add_argument("--target-mode", default="maxsquare", choices=["maxsquare", "IW_maxsquare"])
    ap.add_argument("--multi", default="False")
    ap.add_argument("--lambda-target", type=float, default=0.1)
    ap.add_argument("--num-classes", type=int, default=19)
    ap.add_argument("--conv-math", default="fp32", choices=["fp32", "fp16", "bf16"],
                    help="fp16 / bf16 = BASELINE config 5's fp16 MFMA path (fp16: scaled fp16 operands; fp32 accumulation)")
    ap.add_argument("--bn-form", default="fused", choices=["fused", "split"],
                    help="BN kernels: one fused launch per call (default) or split statistics/apply launches")
    ap.add_argument("--f32-form", default=None, choices=["mfma_f32", "bf16x6", "f16x3"],
                    help="matrix-core form of the fp32 convs (default: the library's)")
    ap.add_argument("--graph", type=int, default=1,
                    help="1: iterations after the first replay one captured hipGraph (single process); 0: eager")
    ap.add_argument("--pair", type=int, default=1,
                    help="1: source and target images run through the network as one image pair (one GEMM per conv "
                         "over both, per-image BN statistics, one backward); 0: two forward/backward passes")
    ap.add_argument("--overlap", type=int, default=1,
                    help="with --pair 0: the target forward runs on a side stream concurrently with the source backward")
    ap.add_argument("--async-wgrad", type=int, default=0,
                    help="1: in-place weight gradients on a side stream beside the data-gradient chain (ops.ASYNC_WGRAD)")
    ap.add_argument("--cpu-baseline-iters", type=int, default=2, help="0 disables the CPU baseline")
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"),
                    help="PMC-derived HBM traffic per launch of the dominant kernel (from a rocprofv3 --pmc run)")
    return ap.parse_args()


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}: launch N>1 with torchrun")
    argv = ["--crop_size", f"{a.width},{a.height}", "--target_crop_size", f"{a.width},{a.height}",
            "--imagenet_pretrained", "False", "--save_dir", "", "--num_classes", str(a.num_classes),
            "--target_mode", a.target_mode, "--multi", a.multi, "--lambda_target", str(a.lambda_target),
            "--iter_max", "200000", "--conv_math", a.conv_math, "--graph", str(bool(a.graph)),
            "--overlap", str(bool(a.overlap)), "--pair", str(bool(a.pair))]
    if a.f32_form:
        argv += ["--f32_form", a.f32_form]
    args, _, _ = init_args(build_parser().parse_args(argv))
    ops.set_bn_fused(a.bn_form == "fused")
    ops.ASYNC_WGRAD = bool(a.async_wgrad)
    tr = UDATrainer(args, cuda=True)
    rank, dev = tr.rank, tr.device
    init_state = {k: v.detach().cpu().clone() for k, v in tr.model.state_dict().items()} if rank == 0 else None

    # inputs resident in HBM before timing: two (source, label, target) triples per rank
    H, W, C = a.height, a.width, a.num_classes
    batches = []
    for i in range(2):
        seed = 1000 * rank + i
        batches.append((synthetic_image(H, W, seed).to(dev), synthetic_labels(H, W, C, seed).to(dev),
                        synthetic_image(H, W, 500 + seed).to(dev)))
    torch.cuda.synchronize()

    h3, w3 = feat_hw(H), feat_hw(W)
    nimg = 2 if tr.pair else 1  # images per layer3 conv call
    key = (1, 256, 256, h3, w3, 2, nimg)
    graphed = bool(tr.use_graph)
    first_losses = None
    for i in range(max(a.warmup, 1 if graphed else 0)):
        tr.uda_step(*batches[i % 2])
        if i == 0:
            first_losses = {"loss_seg": tr.loss_val.detach().clone(), "loss_target": tr.loss_target.detach().clone()}
    torch.cuda.synchronize()
    if not graphed:
        ops.PROBE[key] = []
        if tr.overlap and not tr.pair:  # eager: time the probe's kernel on its own in one sequential iteration below
            ops.PROBE.pop(key)

    if dist.is_initialized():
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        tr.uda_step(*batches[i % 2])
    torch.cuda.synchronize()
    if dist.is_initialized():
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if graphed or key not in ops.PROBE:
        # HIP events cannot time kernels inside a replayed graph: the dominant kernel is timed on
        # one eager iteration right after the timed replays (same shapes, the trained weights).
        # A spin kernel first keeps the GPU busy while the host enqueues that iteration (~35 ms of
        # Python), so its kernels run back to back and the probe's event pairs hold no host gaps.
        try:
            torch.cuda._sleep(int(120e6))  # ~60 ms at the ~2 GHz the chip holds
        except Exception:
            pass
        ops.PROBE[key] = []
        tr.overlap = False  # the probe times the kernel alone, not sharing the GPU with another stream
        tr._uda_body(*batches[0])
        torch.cuda.synchronize()
    probes = ops.PROBE.pop(key)
    kern_ms = sum(s.elapsed_time(e) for s, e in probes) / max(len(probes), 1)

    el = torch.tensor([elapsed], device=dev, dtype=torch.float64)
    if dist.is_initialized():
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = el.item()
    images = 2 * a.steps * world
    if rank != 0:
        dist.destroy_process_group()
        return

    flops = 2.0 * 256 * 256 * 9 * h3 * w3 * nimg
    achieved = flops / (kern_ms * 1e-3) / 1e12
    form = ops.f32_form() if a.conv_math == "fp32" else a.conv_math
    # the op the probe timed: the stream-K GEMM + its piece-reduce launch
    kernels = "k_igemm_fwd_sk,k_sk_reduce"
    traffic, rec = None, None
    if os.path.exists(a.pmc):
        try:
            rec = json.load(open(a.pmc))
        except Exception:
            rec = None
    # the committed PMC figure counts only if it was measured on this very kernel: form, image count,
    # map size and the launches one op call makes
    if rec is not None and (rec.get("form") == form and rec.get("nimg") == nimg and rec.get("h") == h3
                            and rec.get("w") == w3 and rec.get("kernel") == kernels):
        traffic = rec.get("hbm_bytes_per_launch")
    # the bound of the kernel's own arithmetic: FP32 MFMA, BF16 MFMA, or BF16 MFMA at six
    # products per fp32 product (the bf16x6 form): 2500 / 6 = 416.7 fp32-equivalent TFLOP/s
    # and FP16 MFMA (same rate) at three products per fp32 product (the f16x3 form): 833.3
    peak = {"mfma_f32": FP32_MFMA_PEAK_TFLOPS, "bf16": BF16_MFMA_PEAK_TFLOPS, "fp16": BF16_MFMA_PEAK_TFLOPS,
            "bf16x6": round(BF16_MFMA_PEAK_TFLOPS / 6, 1), "f16x3": round(BF16_MFMA_PEAK_TFLOPS / 3, 1)}[form]
    roofline = {"bound": "mfma", "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s",
                "frac": round(achieved / peak, 4), "traffic": traffic,
                "traffic_source": (os.path.relpath(a.pmc, ROOT) + ": committed rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE "
                                   "passes of this kernel (scripts/gpu_bench_prof.sh), not measured in this run; "
                                   "memory-side bytes incl. Infinity-Cache hits") if traffic is not None else None,
                "kernel": f"dconv3x3 fwd layer3 d=2 over {nimg} image(s): one op call = the stream-K GEMM "
                          "k_igemm_fwd_sk(2) + its piece reduce k_sk_reduce (the weight planes are split at pack "
                          "time, once per SGD step; f16x3: the input's absmax partials come from the BN kernel "
                          "that produced it)",
                "form": form, "kernel_ms": round(kern_ms, 4), "launches": len(probes),
                "algorithmic_gflop_per_launch": round(flops / 1e9, 3),
                # NOT a utilisation: fp32-equivalent TFLOP/s of the f16x3 / bf16x6 forms (3 / 6 MFMAs per
                # fp32 product on the FP16 / BF16 pipes) compared with the FP32 matrix pipe's spec
                "fp32_equiv_speedup_vs_fp32_mfma_spec": round(achieved / FP32_MFMA_PEAK_TFLOPS, 4)}

    cpu = None
    loss_delta = None
    if world == 1 and a.cpu_baseline_iters > 0:
        from oracle import msl_oracle as orc
        nthreads = torch.get_num_threads()
        model = orc.Model(init_state, C)
        opt = orc.SGDMult(model.params, model.names, args.lr)
        cfg = dict(lr=args.lr, iter_max=args.iter_max, lambda_seg=args.lambda_seg, IW_ratio=args.IW_ratio,
                   threshold=args.threshold, target_mode=args.target_mode, multi=args.multi,
                   lambda_target=args.lambda_target)
        xs, ys, xt = (t.cpu() for t in batches[0])
        times = []
        for it in range(1 + a.cpu_baseline_iters):
            t1 = time.perf_counter()
            out = orc.uda_step(model, opt, xs, ys, xt, cfg, it)
            times.append(time.perf_counter() - t1)
            if it == 0 and first_losses is not None:
                loss_delta = {k: abs(first_losses[k].item() - out[k]) / max(abs(out[k]), 1e-30)
                              for k in ("loss_seg", "loss_target")}
        s_per_iter = sorted(times[1:])[len(times[1:]) // 2]
        cpu = {"value": round(2.0 / s_per_iter, 4), "unit": "images/s", "cores": nthreads, "kind": "port",
               "sample": f"oracle/msl_oracle.py uda_step at {W}x{H} ({args.target_mode}, multi={args.multi}), "
                         f"median of {a.cpu_baseline_iters} iterations after 1 warm-up, torch-CPU {nthreads} threads",
               "s_per_iter": round(s_per_iter, 3)}

    ms_per_step = elapsed / a.steps * 1e3
    # the whole step against the conv roofline (north_star: "images/sec ... as fraction of the conv
    # roofline"): every conv's algorithmic FLOPs of one iteration (2 images x (forward + data gradient +
    # weight gradient), the stem without its data gradient) over the measured step time
    fwd_gf, stem_gf = conv_gflop(H, W, C)
    step_gf = 2 * (3 * fwd_gf - stem_gf)
    step_tf = step_gf / ms_per_step
    bound = {"f16x3": round(BF16_MFMA_PEAK_TFLOPS / 3, 1), "bf16x6": round(BF16_MFMA_PEAK_TFLOPS / 6, 1),
             "mfma_f32": FP32_MFMA_PEAK_TFLOPS, "fp16": BF16_MFMA_PEAK_TFLOPS, "bf16": BF16_MFMA_PEAK_TFLOPS}[form]
    step_roofline = {"conv_gflop_per_step": round(step_gf, 1), "achieved_tflops": round(step_tf, 2),
                     "frac_of_form_bound": round(step_tf / bound, 4), "form_bound_tflops": bound,
                     "frac_of_fp32_mfma_spec": round(step_tf / FP32_MFMA_PEAK_TFLOPS, 4),
                     "note": "all conv FLOPs of one iteration / ms_per_step; the form bound is the MFMA peak of "
                             "the conv math's form (f16x3: 2500/3 fp32-equivalent TFLOP/s); the FP32 spec "
                             "fraction compares fp32-equivalent work with the FP32 matrix pipe"}
    line = {
        "metric": METRIC, "value": round(images / elapsed, 3), "unit": "images/s", "n_gpus": world,
        "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(ms_per_step, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "fp32" if a.conv_math == "fp32" else f"{a.conv_math} (conv MFMA), fp32",
        "data": "synthetic (counter-generated uint8 images -> BGR-mean, uniform labels; random-init weights)",
        "config": {"workload": f"{'SYNTHIA' if C == 16 else 'GTA5'}->Cityscapes {args.target_mode} UDA step "
                               f"(solve_gta5.py), {W}x{H}, bs=1/GPU",
                   "conv_math": a.conv_math, "bn_form": a.bn_form, "hipgraph": graphed, "pair": bool(a.pair), "overlap": bool(a.overlap), "async_wgrad": bool(a.async_wgrad), "f32_form": ops.f32_form() if a.conv_math == "fp32" else None,
                   "target_mode": args.target_mode, "multi": args.multi, "lambda_target": args.lambda_target,
                   "num_classes": C, "global_batch": 2 * world, "parallelism": f"dp{world}"},
        "roofline": roofline, "step_roofline": step_roofline, "cpu_baseline": cpu,
        "loss_delta_vs_cpu": None if loss_delta is None else {k: float(f"{v:.3g}") for k, v in loss_delta.items()},
        "iterations_per_s": round(a.steps * 1.0 / elapsed, 4),
    }
    print(json.dumps(line), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
