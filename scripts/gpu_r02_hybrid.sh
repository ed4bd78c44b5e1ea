#!/bin/bash
# Hybrid data-parallel + stream-K forward schedule and the coalesced dY split: op tests, the
# per-GEMM 1x1 dispatch timings, bench lines (graph default) and a kernel-trace profile.
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
TAG=${1:-hy}
./scripts/gpu_steps.sh \
  "400|t_$TAG.log|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k 'dconv or pconv or conv1x1 or sk_hybrid or aspp'" \
  "300|d1x1_$TAG.log|python -u scripts/bench_conv1x1_dispatch.py" \
  "300|bench_$TAG.log|python bench.py --cpu-baseline-iters 0" || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o prof --output-format csv -- python3 $R/bench.py --graph 0 --steps 5 --warmup 2 --cpu-baseline-iters 0 > $R/gpurun_out/prof_$TAG.log 2>&1
