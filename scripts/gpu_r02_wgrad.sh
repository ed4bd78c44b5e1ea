#!/bin/bash
# k_wgrad_x6 in the library: op + parity tests, eager bench, kernel-trace profile of the bench.
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
./scripts/gpu_steps.sh \
  "400|t_ops.log|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_parity.py -k 'dconv or pconv or conv1x1 or aspp or conv'" \
  "300|bench_eager.log|python bench.py --graph 0 --cpu-baseline-iters 0" || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_e -o prof --output-format csv -- python3 $R/bench.py --graph 0 --steps 5 --warmup 2 --cpu-baseline-iters 0 > $R/gpurun_out/prof_e.log 2>&1
