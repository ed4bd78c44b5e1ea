#!/bin/bash
# On the GPU box (r05): the KG=2 forward-form GEMMs - the op / pack / parity GPU tests on the new library,
# then a same-box A/B against the base build (maxsquareloss_amd/_lib/base) with per-op timings and bench lines.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-k}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_ops.py tests/test_gpu_parity.py tests/test_gpu_graph.py > gpurun_out/kg2_tests_$TAG.log 2>&1 || exit $?
bash scripts/gpu_ab.sh kg2_$TAG maxsquareloss_amd/_lib/base/libmsl_hip.so maxsquareloss_amd/_lib/libmsl_hip.so
