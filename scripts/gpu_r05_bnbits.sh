#!/bin/bash
# On the GPU box (r05): the BN mask-bits change - its tests, per-call BN timings (with / without the bits)
# and same-box step A/B (ops.BN_MASK_BITS off / on, alternating).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
OUT=gpurun_out/r05_bnbits.log
: > $OUT
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ops.py \
  -k "bn_ or bottleneck" tests/test_gpu_pair.py tests/test_gpu_graph.py >> $OUT 2>&1 || exit $?
timeout -k 10 120 python scripts/bench_bn.py >> $OUT 2>&1 || exit $?
for round in 1 2; do
  for bits in False True; do
    echo "=== BN_MASK_BITS=$bits round $round" >> $OUT
    timeout -k 10 200 python -c "
import sys, runpy
sys.argv = ['bench.py', '--cpu-baseline-iters', '0']
import maxsquareloss_amd.ops as o
o.BN_MASK_BITS = $bits
runpy.run_path('bench.py', run_name='__main__')" 2>/dev/null | grep -o '"ms_per_step": [0-9.]*' >> $OUT || exit $?
  done
done
