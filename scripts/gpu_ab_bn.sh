#!/bin/bash
# On the GPU box: same-box A/B of two builds (MSL_LIB_PATH) on the BN kernels - the BN / pair GPU tests on
# the experiment, then per-call BN timings (scripts/bench_bn.py) and bench lines, alternating twice.
#   scripts/gpu_ab_bn.sh <tag> <base .so> <exp .so>
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=$1; BASE=$2; EXP=$3
cd $R && mkdir -p gpurun_out
MSL_LIB_PATH=$R/$EXP timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_pair.py tests/test_gpu_graph.py tests/test_gpu_ops.py -k "bn or pair or graph or reproducible" \
  > gpurun_out/${TAG}_tests.log 2>&1 || exit $?
OUT=gpurun_out/${TAG}_ab.log
: > $OUT
for round in 1 2; do
  for which in base exp; do
    lib=$BASE; [ $which = exp ] && lib=$EXP
    echo "=== $which round $round ($lib)" >> $OUT
    MSL_LIB_PATH=$R/$lib timeout -k 10 200 python scripts/bench_bn.py >> $OUT 2>&1 || exit $?
    MSL_LIB_PATH=$R/$lib timeout -k 10 200 python bench.py --cpu-baseline-iters 0 2>/dev/null | grep -o '"ms_per_step": [0-9.]*' >> $OUT || exit $?
  done
done
