#!/bin/bash
# On the GPU box (r06 evidence): the -m gpu suite without the full-size configs (every failure reported), smoke(),
# the default bench line (with the CPU baseline) and a rocprofv3 kernel-trace of a short bench run with the
# replayed iteration's breakdown (scripts/replay_breakdown.py).  Logs: gpurun_out/<tag>_*.
#   scripts/gpu_r06_final.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-fin}
O=$R/gpurun_out
cd $R && mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread \
  --deselect tests/test_gpu_configs.py > $O/${TAG}_suite_a.log 2>&1
rc=$?
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc   # 1 = test failures (reported); anything else ends the call
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/${TAG}_smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${TAG}_prof -o prof --output-format csv -- python3 $R/bench.py \
  --steps 5 --warmup 2 --cpu-baseline-iters 0 > $O/${TAG}_prof.log 2>&1 || exit $?
CSV=$(find $O/${TAG}_prof -name '*kernel_trace.csv' | head -n 1)
python3 $R/scripts/replay_breakdown.py $CSV 3 > $O/${TAG}_breakdown.txt
exit $rc
