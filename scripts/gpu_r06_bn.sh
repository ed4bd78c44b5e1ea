#!/bin/bash
# On the GPU box (r06): BN kernel A/B - the BN tests on the tree's library, per-call timings (scripts/bench_bn.py)
# at the 1024x512 (65 x 129) and config-5 (96 x 161) layer3 maps for each library, then bench lines of configs 2
# and 5 alternating the libraries.  Logs: gpurun_out/<tag>_*.
#   scripts/gpu_r06_bn.sh <tag> <lib .so> [<lib .so> ...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
TAG=$1; shift
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_pair.py \
  -k "bn or masked_residual or bottleneck" > gpurun_out/${TAG}_t.log 2>&1 || exit $?
for lib in "$@"; do
  for hw in "65 129" "96 161"; do
    echo "=== $lib $hw" >> gpurun_out/${TAG}_bn.log
    MSL_LIB_PATH=$R/$lib timeout -k 10 200 python scripts/bench_bn.py --hw $hw >> gpurun_out/${TAG}_bn.log 2>&1 || exit $?
  done
done
B="timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-baseline-iters 0"
for round in 1 2; do
  for lib in "$@"; do
    echo "=== $lib round $round" >> gpurun_out/${TAG}_steps.log
    MSL_LIB_PATH=$R/$lib $B 2>/dev/null | grep -o '"ms_per_step": [0-9.]*' >> gpurun_out/${TAG}_steps.log || exit $?
    MSL_LIB_PATH=$R/$lib $B --num-classes 16 --conv-math fp16 --height 760 --width 1280 --target-mode IW_maxsquare \
      --multi True 2>/dev/null | grep -o '"ms_per_step": [0-9.]*' | sed 's/^/cfg5 /' >> gpurun_out/${TAG}_steps.log || exit $?
  done
done
