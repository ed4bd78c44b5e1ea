#!/bin/bash
# f16x3 on the 64- / 32-row tiles: op tests in that form, small-M op A/B, bench
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread \
  -k "f16x3" > gpurun_out/small_tests.log 2>&1 || { tail -40 gpurun_out/small_tests.log; exit 1; }
tail -2 gpurun_out/small_tests.log
timeout -k 10 300 python -u scripts/bench_small_h3.py > gpurun_out/small_ab.jsonl 2>&1 || { tail -20 gpurun_out/small_ab.jsonl; exit 1; }
grep form gpurun_out/small_ab.jsonl
timeout -k 10 300 python -u bench.py --cpu-baseline-iters 0 > gpurun_out/small_bench.json 2>&1 || { tail -20 gpurun_out/small_bench.json; exit 1; }
tail -1 gpurun_out/small_bench.json | cut -c150-240
