#!/bin/bash
# On the GPU box: the conv -> BN fusion tests, then a bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-fold}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fold.py -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --cpu-baseline-iters 0 > gpurun_out/${TAG}_bench.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_prof -o prof --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --cpu-baseline-iters 0 > $R/gpurun_out/${TAG}_prof.log 2>&1
