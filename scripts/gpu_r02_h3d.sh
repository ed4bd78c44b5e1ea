#!/bin/bash
# f16x3 default (BN-fed operand scales): full GPU suite, accuracy table, bench (+ x6 on the same box) and a kernel profile
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  > gpurun_out/h3d_tests.log 2>&1; rc=$?; tail -3 gpurun_out/h3d_tests.log; grep -E 'FAILED|ERROR' gpurun_out/h3d_tests.log | head
[ $rc -le 1 ] || exit 1
timeout -k 10 300 python -u scripts/form_accuracy.py > gpurun_out/h3d_accuracy.txt 2>&1 || { tail gpurun_out/h3d_accuracy.txt; exit 1; }
cat gpurun_out/h3d_accuracy.txt
timeout -k 10 400 python -u bench.py > gpurun_out/h3d_bench.json 2> gpurun_out/h3d_bench.err || { tail -30 gpurun_out/h3d_bench.err; exit 1; }
cat gpurun_out/h3d_bench.json
timeout -k 10 300 python -u bench.py --cpu-baseline-iters 0 --f32-form bf16x6 > gpurun_out/h3d_bench_x6.json 2> gpurun_out/h3d_bench_x6.err || { tail -30 gpurun_out/h3d_bench_x6.err; exit 1; }
cut -c1-400 gpurun_out/h3d_bench_x6.json
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/h3d_prof -o run -- python3 -u bench.py --steps 10 --warmup 3 \
  --cpu-baseline-iters 0 > gpurun_out/h3d_prof_bench.json 2> gpurun_out/h3d_prof_bench.err || { tail -30 gpurun_out/h3d_prof_bench.err; exit 1; }
