#!/bin/bash
# Same-box full-step A/B of the 1x1 dispatch rules (scripts/bench_plan_ab.py), alternating.
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
TAG=${1:-pab}
./scripts/gpu_steps.sh \
  "200|${TAG}_new1.log|python scripts/bench_plan_ab.py new --cpu-baseline-iters 0" \
  "200|${TAG}_old1.log|python scripts/bench_plan_ab.py old --cpu-baseline-iters 0" \
  "200|${TAG}_fwdm1.log|python scripts/bench_plan_ab.py fwdm --cpu-baseline-iters 0" \
  "200|${TAG}_new2.log|python scripts/bench_plan_ab.py new --cpu-baseline-iters 0" \
  "200|${TAG}_old2.log|python scripts/bench_plan_ab.py old --cpu-baseline-iters 0" \
  "200|${TAG}_fwdm2.log|python scripts/bench_plan_ab.py fwdm --cpu-baseline-iters 0" || exit $?
