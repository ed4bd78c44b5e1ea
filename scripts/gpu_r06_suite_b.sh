#!/bin/bash
# On the GPU box (r06 evidence): the full-size config tests (tests/test_gpu_configs.py, every failure reported),
# then the BASELINE configs' bench lines and the layer3 op in the three fp32 forms (scripts/gpu_r06_configs.sh).
#   scripts/gpu_r06_suite_b.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-fin}
cd $R && mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_configs.py -m gpu -v -rf --timeout 600 --timeout-method thread \
  > gpurun_out/${TAG}_suite_b.log 2>&1
rc=$?
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash $R/scripts/gpu_r06_configs.sh $TAG || exit $?
exit $rc
