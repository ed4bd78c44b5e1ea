#!/bin/bash
# On the GPU box (r05): the RCCL one-rank DP test alone, with RCCL's own log, progress to gpurun_out.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
NCCL_DEBUG=INFO timeout -k 10 240 python -u -m pytest -s -v --timeout 200 --timeout-method thread \
  tests/test_gpu_dp.py -k rccl > gpurun_out/r05_rccl.log 2>&1
