#!/bin/bash
# On the GPU box: the -m gpu suite (no -x: every failure reported), smoke(), the default bench line (with
# the CPU baseline) and a rocprofv3 kernel-trace of a short bench run.  TAG names the logs.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-x}
cd $R && mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1
rc=$?
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc   # 1 = test failures (reported); anything else ends the call
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o prof --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --cpu-baseline-iters 0 > $R/gpurun_out/prof_$TAG.log 2>&1 && \
exit $rc
