#!/bin/bash
# On the GPU box: the matrix-core forms of the stream-K conv kernels vs fp64 (tune_dconv x6),
# then the bench line + kernel-trace / PMC profiles of the default path (gpu_bench_prof.sh).
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 ./scripts/tune_dconv x6 > $O/tune_x6.log 2>&1
bash $R/scripts/gpu_bench_prof.sh ${1:-r01s2}
