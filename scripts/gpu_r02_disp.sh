#!/bin/bash
# 1x1 dispatch timings and two bench lines
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
TAG=${1:-disp}
./scripts/gpu_steps.sh \
  "300|d1x1_$TAG.log|python -u scripts/bench_conv1x1_dispatch.py" \
  "300|bench_$TAG.log|python bench.py --cpu-baseline-iters 0" \
  "300|bench2_$TAG.log|python bench.py --cpu-baseline-iters 0" || exit $?
