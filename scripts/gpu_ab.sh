#!/bin/bash
# On the GPU box: same-box A/B of two builds of libmsl_hip.so (MSL_LIB_PATH): per-op GEMM timings at the
# step's pair shapes (scripts/bench_ops.py) and bench lines, alternating base / experiment twice.
#   scripts/gpu_ab.sh <tag> <base .so> <exp .so> [bench_ops --only filter]
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=$1; BASE=$2; EXP=$3; ONLY=${4:-}
cd $R && mkdir -p gpurun_out
OUT=gpurun_out/${TAG}_ab.log
: > $OUT
for round in 1 2; do
  for which in base exp; do
    lib=$BASE; [ $which = exp ] && lib=$EXP
    echo "=== $which round $round ($lib)" >> $OUT
    MSL_LIB_PATH=$R/$lib timeout -k 10 200 python scripts/bench_ops.py --nimg 2 --reps 30 ${ONLY:+--only "$ONLY"} >> $OUT 2>&1 || exit $?
    MSL_LIB_PATH=$R/$lib timeout -k 10 200 python bench.py --cpu-baseline-iters 0 2>/dev/null | grep -o '"ms_per_step": [0-9.]*' >> $OUT || exit $?
  done
done
