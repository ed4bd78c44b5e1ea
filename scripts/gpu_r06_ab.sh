#!/bin/bash
# r06 kernel-form round on the GPU box: fp64 checks of every conv op of the tree's library at the step's pair
# shapes, the conv op tests, the determinism probe, then the same-box A/B of the given builds.
#   scripts/gpu_r06_ab.sh <tag> [--skip-checks] <lib .so> ... [-- bench_ops --only filter]
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
TAG=$1; shift
if [ "$1" = "--skip-checks" ]; then
  shift
else
  timeout -k 10 300 python -u scripts/bench_ops.py --nimg 2 --check --reps 5 > gpurun_out/${TAG}_check.log 2>&1 || exit $?
  timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py \
    -k "dconv_fwd_bwd or f16x3 or conv_fp16_math or wgrad or aspp or launch_guard or pconv or conv1x1 or sk_hybrid or bottleneck or masked_residual" > gpurun_out/${TAG}_tests.log 2>&1 || exit $?
  timeout -k 10 300 python -u scripts/dbg_det.py > gpurun_out/${TAG}_det.log 2>&1 || exit $?
fi
scripts/gpu_ab.sh "$TAG" "$@"
