#!/bin/bash
# On the GPU box (r05): same-box A/B of two library builds on BASELINE configs 4 and 5 (the large-map
# configs): bench lines alternating base / exp twice each.
#   scripts/gpu_r05_cfgab.sh <tag> <base .so> <exp .so>
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=$1; BASE=$2; EXP=$3
cd $R && mkdir -p gpurun_out
OUT=gpurun_out/${TAG}_cfgab.log
: > $OUT
C4="--target-mode IW_maxsquare --multi True --lambda-target 0.09 --height 640 --width 1280"
C5="--num-classes 16 --conv-math fp16 --height 760 --width 1280 --target-mode IW_maxsquare --multi True"
for cfg in 4 5; do
  args=$C4; [ $cfg = 5 ] && args=$C5
  for round in 1 2; do
    for which in base exp; do
      lib=$BASE; [ $which = exp ] && lib=$EXP
      echo "=== config $cfg $which round $round ($lib)" >> $OUT
      MSL_LIB_PATH=$R/$lib timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-baseline-iters 0 $args 2>/dev/null | grep -o '"ms_per_step": [0-9.]*' >> $OUT || exit $?
    done
  done
done
