#!/bin/bash
# On the GPU box (r05): per-kernel step profile with the BN mask bits off / on (rocprofv3 kernel trace of
# bench.py via scripts/bench_with.py), plus the BN per-call timings.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
OUT=gpurun_out/r05_bnbits2.log
: > $OUT
timeout -k 10 120 python scripts/bench_bn.py >> $OUT 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
for bits in False True; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/bits_$bits -o run -- \
    python3 $R/scripts/bench_with.py ops.BN_MASK_BITS=$bits -- --steps 5 --warmup 2 --cpu-baseline-iters 0 \
    >> $R/$OUT 2>&1 || exit $?
done
