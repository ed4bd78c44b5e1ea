#!/bin/bash
# BN split-form absmax test, then the 1x1 per-GEMM dispatch table in the f16x3 form
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -v --timeout 200 --timeout-method thread -k "absmax or bn_act" \
  > gpurun_out/h3e_tests.log 2>&1 || { tail -40 gpurun_out/h3e_tests.log; exit 1; }
tail -2 gpurun_out/h3e_tests.log
timeout -k 10 400 python -u scripts/bench_conv1x1_dispatch.py --form f16x3 > gpurun_out/h3e_disp.txt 2>&1 || { tail -20 gpurun_out/h3e_disp.txt; exit 1; }
cat gpurun_out/h3e_disp.txt
