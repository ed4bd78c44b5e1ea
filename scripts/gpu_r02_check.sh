#!/bin/bash
# quick check after a kernel-layout change: f16x3 / fp16 / bf16 op + parity tests
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread \
  -k "f16x3 or fp16 or bf16" > gpurun_out/chk_tests.log 2>&1 || { tail -40 gpurun_out/chk_tests.log; exit 1; }
tail -2 gpurun_out/chk_tests.log
