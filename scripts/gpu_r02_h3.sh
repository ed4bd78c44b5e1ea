#!/bin/bash
# f16x3 form: op tests in that form + the accuracy test, then a same-box A/B of the GEMM shapes
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -x -v --timeout 120 --timeout-method thread -k "f16x3 or pconv or dconv" \
  > gpurun_out/h3_tests.log 2>&1 || { tail -50 gpurun_out/h3_tests.log; exit 1; }
tail -3 gpurun_out/h3_tests.log
timeout -k 10 300 python -u scripts/bench_forms.py bf16x6,f16x3 > gpurun_out/h3_forms.jsonl 2>&1 || { tail -30 gpurun_out/h3_forms.jsonl; exit 1; }
cat gpurun_out/h3_forms.jsonl
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/h3_prof -o run -- python -u scripts/bench_forms.py f16x3 > gpurun_out/h3_prof.log 2>&1 || { tail -30 gpurun_out/h3_prof.log; exit 1; }
find gpurun_out/h3_prof -name '*kernel_stats.csv' | head -1 | xargs head -30
