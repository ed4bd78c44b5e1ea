#!/bin/bash
# On the GPU box (r05): the dominant op's counters (FETCH/WRITE traffic, two SQ passes) and the
# bench lines of the BASELINE configs (2, 4, 5 and the bf16 variant of 2).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
bash scripts/gpu_counters.sh r05dom k_igemm_fwd_sk,k_sk_reduce $R/scripts/prof_dominant.py 20 || exit $?
cd $R && GRAFT_REPO_ROOT=$R bash scripts/gpu_configs.sh || exit $?
