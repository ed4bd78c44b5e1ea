#!/bin/bash
# On the GPU box (r05): a kernel-trace profile of the default bench (5 steps) and the kernel-time
# breakdown of one replayed iteration (scripts/replay_breakdown.py).  Extra arguments go to bench.py.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-bd}
shift
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$TAG -o prof --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --cpu-baseline-iters 0 "$@" > $O/prof_$TAG.log 2>&1 || exit $?
CSV=$(find $O/prof_$TAG -name '*kernel_trace.csv' | head -n 1)
python3 $R/scripts/replay_breakdown.py $CSV 3 > $O/breakdown_$TAG.txt
