#!/bin/bash
# On the GPU box: same-box A/B of two builds of libmsl_hip.so (MSL_LIB_PATH) on the config-4/5 bench
# lines (scripts/gpu_configs.sh arguments), alternating base / experiment twice.
#   scripts/gpu_cfg_ab.sh <tag> <base .so> <exp .so>
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=$1; BASE=$2; EXP=$3
cd $R && mkdir -p gpurun_out
OUT=gpurun_out/${TAG}_cfgab.log
: > $OUT
C4="--target-mode IW_maxsquare --multi True --lambda-target 0.09 --height 640 --width 1280"
C5="--num-classes 16 --conv-math fp16 --height 760 --width 1280 --target-mode IW_maxsquare --multi True"
for round in 1 2; do
  for which in base exp; do
    lib=$BASE; [ $which = exp ] && lib=$EXP
    for c in 4 5; do
      args=$C4; [ $c = 5 ] && args=$C5
      echo "=== cfg$c $which round $round" >> $OUT
      MSL_LIB_PATH=$R/$lib timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-baseline-iters 0 $args 2>/dev/null | grep -o '"ms_per_step": [0-9.]*' >> $OUT || exit $?
    done
  done
done
