#!/bin/bash
# On the GPU box (r05): same-box A/B of two builds on the layer1-sized shapes (129 x 257 pair maps) and
# the bench step, alternating base / exp twice.   scripts/gpu_r05_l1ab.sh <tag> <base .so> <exp .so>
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=$1; BASE=$2; EXP=$3
cd $R && mkdir -p gpurun_out
OUT=gpurun_out/${TAG}_ab.log
: > $OUT
for round in 1 2; do
  for which in base exp; do
    lib=$BASE; [ $which = exp ] && lib=$EXP
    echo "=== $which round $round ($lib)" >> $OUT
    for f in "layer1" "1x1 256->64" "1x1 64->256"; do
      MSL_LIB_PATH=$R/$lib timeout -k 10 200 python scripts/bench_ops.py --nimg 2 --hw 129 257 --reps 30 --only "$f" --which wgrad >> $OUT 2>&1 || exit $?
    done
    MSL_LIB_PATH=$R/$lib timeout -k 10 200 python bench.py --cpu-baseline-iters 0 2>/dev/null | grep -o '"ms_per_step": [0-9.]*' >> $OUT || exit $?
  done
done
