#!/bin/bash
# On the GPU box (r05): the -m gpu suite in two parts (a: everything but the full-size configs; b: the
# full-size configs incl. the config-5 fp16 envelope / loss curve, then smoke and the default bench line).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
PART=${1:-a}; TAG=${2:-s}
cd $R && mkdir -p gpurun_out
if [ "$PART" = a ]; then
  timeout -k 10 1000 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests \
    --deselect tests/test_gpu_configs.py > gpurun_out/suite_a_$TAG.log 2>&1
  exit $?
fi
timeout -k 10 800 python -u -m pytest -s -v --timeout 700 --timeout-method thread -m gpu \
  tests/test_gpu_configs.py > gpurun_out/suite_b_$TAG.log 2>&1
rc=$?
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit $?
timeout -k 10 200 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
exit $rc
