#!/bin/bash
# On the GPU box: run one named step (or several) with its own time limit; logs under gpurun_out/.
#   tests [pytest-args]   the -m gpu suite (no -x: every failure is reported)
#   smoke                 __graft_entry__.smoke()
#   bench [args]          bench.py
#   py <script> [args]    any python script
#   prof [bench args]     rocprofv3 kernel trace + stats of a short bench run
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${TAG:-x}
cd $R && mkdir -p gpurun_out
step=$1; shift
case $step in
  tests) timeout -k 10 ${T:-900} python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread "$@" > gpurun_out/tests_$TAG.log 2>&1 ;;
  smoke) timeout -k 10 ${T:-300} python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 ;;
  bench) timeout -k 10 ${T:-400} python -u bench.py "$@" > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err ;;
  py) timeout -k 10 ${T:-600} python -u "$@" > gpurun_out/py_$TAG.log 2>&1 ;;
  prof) cd /tmp && export TMPDIR=/tmp && timeout -k 10 ${T:-400} rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o prof --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --cpu-baseline-iters 0 "$@" > $R/gpurun_out/prof_$TAG.log 2>&1 ;;
  *) echo "unknown step $step"; exit 2 ;;
esac
