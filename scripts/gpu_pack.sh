#!/bin/bash
# Pack-kernel A/B under a kernel trace, the pack/conv op tests, then the bench + step profile.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "pack or conv" -x -q --timeout 120 --timeout-method thread > gpurun_out/pack_tests.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 200 rocprofv3 --kernel-trace -d $R/gpurun_out/profpack -o prof --output-format csv -- python3 $R/scripts/pack_bench.py > $R/gpurun_out/profpack.log 2>&1 && \
cd $R && bash scripts/gpu_round.sh pk2
