#!/bin/bash
# On the GPU box (r05): where the weight-gradient op's time goes - a kernel-trace of the op alone
# (split, GEMM, reduce) on three shapes, then the SQ counter passes of k_wgrad_x6 on the 1x1 1024->256 one.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for sh in "1x1 1024->256" "layer3 3x3 d2" "1x1 256->1024"; do
  tg=$(echo "$sh" | tr -c 'a-z0-9' '_')
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/wgk_$tg -o k --output-format csv -- python3 $R/scripts/bench_ops.py --nimg 2 --reps 20 --only "$sh" --which wgrad > $O/wgk_$tg.log 2>&1 || exit $?
done
bash $R/scripts/gpu_counters.sh wgsq k_wgrad_x6,k_split_rows,k_wsk_reduce $R/scripts/bench_ops.py --nimg 2 --reps 20 --only "1x1 1024->256" --which wgrad
