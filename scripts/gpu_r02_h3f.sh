#!/bin/bash
# the f16x3 1x1 plan: conv1x1 tests, bench (+ one without the CPU baseline), step kernel profile
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -x -v --timeout 200 --timeout-method thread \
  -k "conv1x1 or residual or model" > gpurun_out/h3f_tests.log 2>&1 || { tail -40 gpurun_out/h3f_tests.log; exit 1; }
tail -2 gpurun_out/h3f_tests.log
timeout -k 10 400 python -u bench.py > gpurun_out/h3f_bench.json 2> gpurun_out/h3f_bench.err || { tail -30 gpurun_out/h3f_bench.err; exit 1; }
cat gpurun_out/h3f_bench.json
timeout -k 10 300 python -u bench.py --cpu-baseline-iters 0 > gpurun_out/h3f_bench2.json 2> gpurun_out/h3f_bench2.err || { tail -30 gpurun_out/h3f_bench2.err; exit 1; }
cut -c1-300 gpurun_out/h3f_bench2.json
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/h3f_prof -o run -- python3 -u bench.py --steps 10 --warmup 3 \
  --cpu-baseline-iters 0 > gpurun_out/h3f_prof_bench.json 2> gpurun_out/h3f_prof_bench.err || { tail -30 gpurun_out/h3f_prof_bench.err; exit 1; }
