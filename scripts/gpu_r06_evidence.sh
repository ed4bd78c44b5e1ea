#!/bin/bash
# On the GPU box (r06): the -m gpu suite without the full-size configs, then a kernel-trace breakdown of one
# replayed iteration of the default bench (scripts/replay_breakdown.py) and the weight-gradient family's SQ
# counters (LDS bank conflicts after the r06 padding) on the 1x1 1024 -> 256 and layer3 shapes.
#   scripts/gpu_r06_evidence.sh <tag> [--no-suite]
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-ev}
O=$R/gpurun_out
mkdir -p $O
cd $R
if [ "$2" != "--no-suite" ]; then
  timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests \
    --deselect tests/test_gpu_configs.py > $O/suite_a_$TAG.log 2>&1 || exit $?
fi
bash $R/scripts/gpu_r05_breakdown.sh $TAG || exit $?
cd /tmp && export TMPDIR=/tmp
bash $R/scripts/gpu_counters.sh wg_$TAG k_wgrad_x6,k_split_rows,k_wsk_reduce $R/scripts/bench_ops.py --nimg 2 --reps 20 \
  --only "1x1 1024->256" --which wgrad || exit $?
bash $R/scripts/gpu_counters.sh wg3_$TAG k_wgrad_x6,k_split_rows,k_wsk_reduce $R/scripts/bench_ops.py --nimg 2 --reps 20 \
  --only "layer3" --which wgrad
