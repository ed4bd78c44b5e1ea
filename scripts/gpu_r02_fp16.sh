#!/bin/bash
# fp16 conv math: op tests, bf16 tests (unchanged path), then config 5 / bf16 vs fp16 bench lines
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -x -v --timeout 200 --timeout-method thread \
  -k "fp16_math or bf16_math" > gpurun_out/fp16_tests.log 2>&1 || { tail -40 gpurun_out/fp16_tests.log; exit 1; }
tail -2 gpurun_out/fp16_tests.log
for m in bf16 fp16; do
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-baseline-iters 0 --num-classes 16 --conv-math $m --height 760 --width 1280 --target-mode IW_maxsquare --multi True > gpurun_out/cfg5_$m.log 2>&1 || { tail -20 gpurun_out/cfg5_$m.log; exit 1; }
  echo "cfg5 $m $(tail -1 gpurun_out/cfg5_$m.log | cut -c150-200)"
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-baseline-iters 0 --conv-math $m > gpurun_out/cfg2_$m.log 2>&1 || { tail -20 gpurun_out/cfg2_$m.log; exit 1; }
  echo "cfg2 $m $(tail -1 gpurun_out/cfg2_$m.log | cut -c150-200)"
done
