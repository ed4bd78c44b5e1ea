#!/bin/bash
# On the GPU box: the ASPP head alone (scripts/prof_aspp.py 20) under a kernel trace, then its counter
# passes (scripts/gpu_counters.sh).  Outputs gpurun_out/<tag>_*.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-aspp}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_trace -o trace --output-format csv -- python3 $R/scripts/prof_aspp.py 20 > $R/gpurun_out/${TAG}_trace.log 2>&1 || exit $?
bash $R/scripts/gpu_counters.sh $TAG k_igemm_fwd_sk2,k_wgrad_x6,k_sk_reduce,k_wsk_reduce $R/scripts/prof_aspp.py 20
