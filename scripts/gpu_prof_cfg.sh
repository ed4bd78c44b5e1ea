#!/bin/bash
# On the GPU box: kernel-trace profiles of the bench step at the headline config and config 5.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-cfg}
cd $R && mkdir -p gpurun_out
C5="--num-classes 16 --conv-math fp16 --height 760 --width 1280 --target-mode IW_maxsquare --multi True"
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_c2prof -o prof --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --cpu-baseline-iters 0 > $R/gpurun_out/${TAG}_c2prof.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_c5prof -o prof --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --cpu-baseline-iters 0 $C5 > $R/gpurun_out/${TAG}_c5prof.log 2>&1
