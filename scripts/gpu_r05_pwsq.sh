#!/bin/bash
# On the GPU box (r05): SQ counters of the forward-form GEMMs alone - the pointwise 256->1024 forward and the
# layer3 3x3 d2 forward over the pair (scripts/gpu_counters.sh passes, bench_ops.py --which fwd).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
bash $R/scripts/gpu_counters.sh pwsq k_igemm_fwd_sk2,k_sk_reduce $R/scripts/bench_ops.py --nimg 2 --reps 20 --only "1x1 256->1024" --which fwd || exit $?
bash $R/scripts/gpu_counters.sh bdsq k_igemm_fwd_sk2,k_sk_reduce $R/scripts/bench_ops.py --nimg 2 --reps 20 --only "layer3" --which fwd
