#!/bin/bash
# the two reworked tests, then per-kernel step profiles of both fp32 forms on one box
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_graph.py -x -v --timeout 200 --timeout-method thread \
  -k "pack_batch or graph_replay" > gpurun_out/h3c_tests.log 2>&1 || { tail -40 gpurun_out/h3c_tests.log; exit 1; }
tail -2 gpurun_out/h3c_tests.log
export TMPDIR=/tmp
for form in bf16x6 f16x3; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/h3c_prof_$form -o run -- python3 -u bench.py --steps 10 --warmup 3 \
    --cpu-baseline-iters 0 --f32-form $form > gpurun_out/h3c_bench_$form.json 2> gpurun_out/h3c_bench_$form.err \
    || { tail -30 gpurun_out/h3c_bench_$form.err; exit 1; }
  tail -1 gpurun_out/h3c_bench_$form.json | cut -c1-300
done
