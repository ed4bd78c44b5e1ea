#!/bin/bash
# Same-box A/B of the BN kernel forms in the bench step (alternating runs), after the BN op tests.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k bn_act -x -q --timeout 120 --timeout-method thread > gpurun_out/bnab_tests.log 2>&1 || exit 1
for i in 1 2; do
  for f in split fused; do
    timeout -k 10 300 python bench.py --cpu-baseline-iters 0 --bn-form $f > gpurun_out/bnab_${f}_$i.log 2>&1 || exit 1
  done
done
