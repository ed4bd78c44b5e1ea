#!/bin/bash
# On the GPU box: evidence for the bench's dominant op (layer3 3x3 d=2 forward over the image pair):
# kernel-trace stats of the probe, then the counter passes (scripts/gpu_counters.sh); then the
# BASELINE config bench lines (scripts/gpu_configs.sh).  TAG names the outputs.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-ev}
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/${TAG}_stats -o stats --output-format csv -- python3 $R/scripts/prof_dominant.py 20 > $O/${TAG}_stats.log 2>&1 || exit $?
bash $R/scripts/gpu_counters.sh $TAG k_igemm_fwd_sk,k_sk_reduce $R/scripts/prof_dominant.py 20 || exit $?
cd $R && bash scripts/gpu_configs.sh
