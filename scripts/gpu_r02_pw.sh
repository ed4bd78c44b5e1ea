#!/bin/bash
# dwordx4 B DMAs for the f16x3 pointwise GEMMs: tests, op A/B, bench A/B on one box
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -v --timeout 200 --timeout-method thread \
  -k "f16x3 and (pconv or conv1x1 or hybrid or residual)" > gpurun_out/pw_tests.log 2>&1 || { tail -40 gpurun_out/pw_tests.log; exit 1; }
tail -2 gpurun_out/pw_tests.log
for v in 0 1 0 1; do
  echo "== MSL_PW_DMA=$v"
  MSL_PW_DMA=$v timeout -k 10 200 python -u scripts/bench_forms.py f16x3 > gpurun_out/pw_$v.jsonl 2>&1 || { tail -20 gpurun_out/pw_$v.jsonl; exit 1; }
  grep '"op": "pw' gpurun_out/pw_$v.jsonl | tail -3 | python3 -c "import sys,json
for l in sys.stdin:
  d=json.loads(l); print(d['op'], 'fwd', d['fwd_us'], 'dgrad', d['dgrad_us'])"
done
for v in 0 1; do
  MSL_PW_DMA=$v timeout -k 10 300 python -u bench.py --cpu-baseline-iters 0 > gpurun_out/pw_bench_$v.json 2>&1 || { tail -20 gpurun_out/pw_bench_$v.json; exit 1; }
  echo "bench MSL_PW_DMA=$v $(tail -1 gpurun_out/pw_bench_$v.json | cut -c150-230)"
done
