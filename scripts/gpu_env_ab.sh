#!/bin/bash
# On the GPU box: same-box A/B of environment settings of one build: per-op GEMM timings at the step's
# pair shapes (scripts/bench_ops.py) and the default bench line, each setting run twice, alternating.
#   scripts/gpu_env_ab.sh <tag> "<env A>" "<env B>" ["<env C>" ...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=$1; shift
cd $R && mkdir -p gpurun_out
OUT=gpurun_out/${TAG}_envab.log
: > $OUT
for round in 1 2; do
  for envs in "$@"; do
    echo "=== [$envs] round $round" >> $OUT
    env $envs timeout -k 10 200 python scripts/bench_ops.py --nimg 2 --reps 30 >> $OUT 2>&1 || exit $?
    env $envs timeout -k 10 200 python bench.py --cpu-baseline-iters 0 2>/dev/null | grep -o '"ms_per_step": [0-9.]*' >> $OUT || exit $?
  done
done
