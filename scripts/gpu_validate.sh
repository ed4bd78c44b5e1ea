#!/bin/bash
# On the GPU box: GPU parity tests, the driver's smoke(), and the default bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/tests_val.log 2>&1 && \
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_val.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/bench_val.log 2>&1
