#!/bin/bash
# On the GPU box: same-box A/B of builds of libmsl_hip.so (MSL_LIB_PATH): per-op GEMM timings at the step's
# pair shapes (scripts/bench_ops.py) and bench lines, alternating the builds, two rounds.
#   scripts/gpu_ab.sh <tag> <lib .so> <lib .so> [more .so ...] [-- bench_ops --only filter]
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=$1; shift
LIBS=()
ONLY=
while [ $# -gt 0 ]; do
  if [ "$1" = "--" ]; then ONLY=$2; break; fi
  LIBS+=("$1"); shift
done
cd $R && mkdir -p gpurun_out
OUT=gpurun_out/${TAG}_ab.log
: > $OUT
for round in 1 2; do
  for lib in "${LIBS[@]}"; do
    echo "=== $lib round $round" >> $OUT
    MSL_LIB_PATH=$R/$lib timeout -k 10 200 python scripts/bench_ops.py --nimg 2 --reps 30 ${ONLY:+--only "$ONLY"} >> $OUT 2>&1 || exit $?
    MSL_LIB_PATH=$R/$lib timeout -k 10 200 python bench.py --cpu-baseline-iters 0 2>/dev/null | grep -o '"ms_per_step": [0-9.]*' >> $OUT || exit $?
  done
done
