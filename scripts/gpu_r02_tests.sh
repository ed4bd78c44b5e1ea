#!/bin/bash
# Full GPU test suite, smoke, bench lines and the 1x1 dispatch timings.
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
TAG=${1:-t}
./scripts/gpu_steps.sh \
  "300|bench_$TAG.log|python bench.py --cpu-baseline-iters 0" \
  "900|gpu_tests_$TAG.log|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "200|smoke_$TAG.log|python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "300|d1x1_$TAG.log|python -u scripts/bench_conv1x1_dispatch.py" \
  "300|bench2_$TAG.log|python bench.py --cpu-baseline-iters 0" || exit $?
