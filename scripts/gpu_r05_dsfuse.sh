#!/bin/bash
# On the GPU box (r05): the RCCL one-rank DP test, the fused residual / downsample gradient tests, and
# a same-box step A/B of the downsample-gradient fusion (deeplab_multi.FUSE_DOWNSAMPLE_GRAD off / on).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
OUT=gpurun_out/r05_dsfuse.log
: > $OUT
timeout -k 10 500 python -u -m pytest -v --timeout 350 --timeout-method thread tests/test_gpu_dp.py -k rccl \
  tests/test_gpu_ops.py::test_bottleneck_fused_residual_grad >> $OUT 2>&1 || exit $?
for round in 1 2; do
  for f in False True; do
    echo "=== FUSE_DOWNSAMPLE_GRAD=$f round $round" >> $OUT
    timeout -k 10 200 python scripts/bench_with.py graphs.models.deeplab_multi.FUSE_DOWNSAMPLE_GRAD=$f -- \
      --cpu-baseline-iters 0 2>/dev/null | grep -o '"ms_per_step": [0-9.]*' >> $OUT || exit $?
  done
done
