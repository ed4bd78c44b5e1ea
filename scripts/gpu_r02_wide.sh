#!/bin/bash
# piece-parallel wgrad reduce for few-tile shapes: tests, then the step bench and its kernel profile
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -x -v --timeout 200 --timeout-method thread \
  -k "pconv or conv1x1 or model" > gpurun_out/wide_tests.log 2>&1 || { tail -40 gpurun_out/wide_tests.log; exit 1; }
tail -2 gpurun_out/wide_tests.log
timeout -k 10 300 python -u bench.py --cpu-baseline-iters 0 > gpurun_out/wide_bench.json 2>&1 || { tail -20 gpurun_out/wide_bench.json; exit 1; }
tail -1 gpurun_out/wide_bench.json | cut -c150-240
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/wide_prof -o run -- python3 -u bench.py --steps 10 --warmup 3 \
  --cpu-baseline-iters 0 > gpurun_out/wide_prof_bench.json 2> gpurun_out/wide_prof_bench.err || { tail -30 gpurun_out/wide_prof_bench.err; exit 1; }
