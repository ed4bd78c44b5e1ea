#!/bin/bash
# Batched weight packs: pack tests, graph / DP / parity tests, bench lines.
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
./scripts/gpu_steps.sh \
  "600|t_pack.log|python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_graph.py tests/test_gpu_dp.py tests/test_gpu_parity.py tests/test_gpu_model.py -k 'pack or graph or dp or source_step or uda'" \
  "300|bench_pk.log|python bench.py --cpu-baseline-iters 0" \
  "300|bench_pk_eager.log|python bench.py --graph 0 --cpu-baseline-iters 0" || exit $?
