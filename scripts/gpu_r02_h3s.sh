#!/bin/bash
# H3S (B split once per workgroup) vs H3P: tests with H3S on, op A/B, bench A/B on one box
mkdir -p gpurun_out
MSL_H3S=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread \
  -k "f16x3 and (dconv or aspp or kat or accurate or hybrid)" > gpurun_out/h3s_tests.log 2>&1 || { tail -40 gpurun_out/h3s_tests.log; exit 1; }
tail -2 gpurun_out/h3s_tests.log
for v in 0 1 0 1; do
  echo "== MSL_H3S=$v"
  MSL_H3S=$v timeout -k 10 200 python -u scripts/bench_forms.py f16x3 > gpurun_out/h3s_$v.jsonl 2>&1 || { tail -20 gpurun_out/h3s_$v.jsonl; exit 1; }
  grep '"op": "layer' gpurun_out/h3s_$v.jsonl | tail -2 | python3 -c "import sys,json
for l in sys.stdin:
  d=json.loads(l); print(d['op'], 'fwd', d['fwd_us'], 'dgrad', d['dgrad_us'])"
done
for v in 0 1 0 1; do
  MSL_H3S=$v timeout -k 10 300 python -u bench.py --cpu-baseline-iters 0 > gpurun_out/h3s_bench_$v.json 2>&1 || { tail -20 gpurun_out/h3s_bench_$v.json; exit 1; }
  echo "bench MSL_H3S=$v $(tail -1 gpurun_out/h3s_bench_$v.json | cut -c150-200)"
done
