#!/bin/bash
# Same-box full-step A/B: current 1x1 rules vs the swapped-operand wgrads on hipBLASLt, alternating.
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
TAG=${1:-pab2}
./scripts/gpu_steps.sh \
  "200|${TAG}_new1.log|python scripts/bench_plan_ab.py new --cpu-baseline-iters 0" \
  "200|${TAG}_wgold1.log|python scripts/bench_plan_ab.py wgold --cpu-baseline-iters 0" \
  "200|${TAG}_new2.log|python scripts/bench_plan_ab.py new --cpu-baseline-iters 0" \
  "200|${TAG}_wgold2.log|python scripts/bench_plan_ab.py wgold --cpu-baseline-iters 0" \
  "200|${TAG}_new3.log|python scripts/bench_plan_ab.py new --cpu-baseline-iters 0" \
  "200|${TAG}_wgold3.log|python scripts/bench_plan_ab.py wgold --cpu-baseline-iters 0" || exit $?
