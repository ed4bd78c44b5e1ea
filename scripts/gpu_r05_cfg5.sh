#!/bin/bash
# On the GPU box (r05): the config-5 fp16 envelope tests (printed margins), then per-op GEMM timings at
# the step's pair shapes (scripts/bench_ops.py) for the kernel work that follows.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-c}
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -s -v --timeout 800 --timeout-method thread -m gpu \
  tests/test_gpu_configs.py -k "cfg5 or config5" > gpurun_out/cfg5_$TAG.log 2>&1
rc=$?
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python scripts/bench_ops.py --nimg 2 --reps 30 > gpurun_out/ops_$TAG.log 2>&1 || exit $?
exit $rc
