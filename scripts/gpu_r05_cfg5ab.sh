#!/bin/bash
# On the GPU box (r05): same-box A/B of two library builds on BASELINE config 5 (fp16 conv math, 1280x760,
# 16 classes, IW_maxsquare, multi) and the default config: bench lines alternating base / exp twice.
#   scripts/gpu_r05_cfg5ab.sh <tag> <base .so> <exp .so>
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=$1; BASE=$2; EXP=$3
cd $R && mkdir -p gpurun_out
OUT=gpurun_out/${TAG}_cfg5ab.log
: > $OUT
for round in 1 2; do
  for which in base exp; do
    lib=$BASE; [ $which = exp ] && lib=$EXP
    echo "=== $which round $round ($lib)" >> $OUT
    MSL_LIB_PATH=$R/$lib timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-baseline-iters 0 --num-classes 16 --conv-math fp16 --height 760 --width 1280 --target-mode IW_maxsquare --multi True 2>/dev/null | grep -o '"ms_per_step": [0-9.]*' >> $OUT || exit $?
  done
done
