#!/bin/bash
# graph test alone, full GPU suite (every form) without it, then a same-box bench A/B of the fp32 forms
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/h3b_graph.log 2>&1; echo "graph test alone: rc $?"; tail -3 gpurun_out/h3b_graph.log
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "not graph_replay" \
  > gpurun_out/h3b_tests.log 2>&1; rc=$?; tail -3 gpurun_out/h3b_tests.log; grep -E 'FAILED|ERROR' gpurun_out/h3b_tests.log | head
[ $rc -le 1 ] || exit 1
for form in bf16x6 f16x3 bf16x6 f16x3; do
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-baseline-iters 0 --f32-form $form \
    > gpurun_out/h3b_bench_$form.json 2> gpurun_out/h3b_bench_$form.err || { tail -30 gpurun_out/h3b_bench_$form.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/h3b_bench_$form.json'));print('$form', d['ms_per_step'], d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
done
