#!/bin/bash
# On the GPU box: selected GPU tests (pytest -k filter $2, or all of tests/ -m gpu when empty), a bench
# line and a kernel-trace profile of the bench.  TAG ($1) names the outputs under gpurun_out/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-r4}
FILT=${2:-}
cd $R && mkdir -p gpurun_out
if [ -n "$FILT" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "$FILT" > gpurun_out/${TAG}_tests.log 2>&1
else
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
fi
rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/${TAG}_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 5 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --cpu-baseline-iters 0 > gpurun_out/${TAG}_bench.log 2>&1 || exit $?
tail -c 600 gpurun_out/${TAG}_bench.log
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_prof -o prof --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --cpu-baseline-iters 0 > $R/gpurun_out/${TAG}_prof.log 2>&1
