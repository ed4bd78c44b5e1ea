#!/bin/bash
# accumulate epilogue: op tests of the accumulating / hybrid paths, then the 1x1 dispatch timings
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
TAG=${1:-acc}
./scripts/gpu_steps.sh \
  "300|t_$TAG.log|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k 'accumulate or sk_hybrid or fused_residual or pconv_fwd'" \
  "300|d1x1_$TAG.log|python -u scripts/bench_conv1x1_dispatch.py" || exit $?
