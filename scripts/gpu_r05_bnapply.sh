#!/bin/bash
# On the GPU box (r05): the cost of a BN-apply in the BD forward's image split (probe PROF 16) at the
# layer3 / layer2 3x3 pair shapes, and the BN kernels (fused, and the stats + apply split) per call.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
OUT=gpurun_out/r05_bnapply.log
[ "$1" = bn ] && OUT=gpurun_out/r05_bnapply_bn.log
: > $OUT
if [ "$1" != bn ]; then
timeout -k 10 120 python scripts/probe_sk.py 256 256 65 129 2 2 >> $OUT 2>&1 || exit $?
timeout -k 10 120 python scripts/probe_sk.py 128 128 65 129 2 1 >> $OUT 2>&1 || exit $?
timeout -k 10 120 python scripts/probe_sk.py 512 512 65 129 2 4 >> $OUT 2>&1 || exit $?
fi
timeout -k 10 120 python scripts/bench_bn.py >> $OUT 2>&1 || exit $?
timeout -k 10 120 python scripts/bench_bn.py --unfused >> $OUT 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/bnprof -o bn -- python $R/scripts/bench_bn.py --unfused --reps 20 > /dev/null 2>&1 || exit $?
find $R/gpurun_out/bnprof -name "*kernel_stats.csv" -exec cp {} $R/gpurun_out/r05_bn_unfused_kernel_stats.csv \;
