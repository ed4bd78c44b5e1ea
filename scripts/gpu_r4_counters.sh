#!/bin/bash
# On the GPU box: r04 counter evidence - the dominant op (layer3 3x3 d=2 forward over the image pair:
# kernel-trace stats, then the FETCH/WRITE/SQ passes of scripts/gpu_counters.sh) and every kernel of the
# UDA step (scripts/gpu_pmc_step.sh).  TAG names the outputs under gpurun_out/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-r04}
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/${TAG}dom_stats -o stats --output-format csv -- python3 $R/scripts/prof_dominant.py 20 > $O/${TAG}dom_stats.log 2>&1 || exit $?
bash $R/scripts/gpu_counters.sh ${TAG}dom k_igemm_fwd_sk,k_sk_reduce $R/scripts/prof_dominant.py 20 || exit $?
bash $R/scripts/gpu_pmc_step.sh $TAG || exit $?
