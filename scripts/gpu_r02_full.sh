#!/bin/bash
# Full GPU test suite, smoke, eager and graph bench lines, kernel-trace profile of the eager bench.
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
./scripts/gpu_steps.sh \
  "900|gpu_tests.log|python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu" \
  "200|smoke.log|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "300|bench_eager.log|python bench.py --graph 0 --cpu-baseline-iters 0" \
  "300|bench_graph.log|python bench.py --graph 1 --cpu-baseline-iters 0" || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_e -o prof --output-format csv -- python3 $R/bench.py --graph 0 --steps 5 --warmup 2 --cpu-baseline-iters 0 > $R/gpurun_out/prof_e.log 2>&1
