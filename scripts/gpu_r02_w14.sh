#!/bin/bash
# f16x3 forward wave layout: 2x2 (each wave 64x64) vs 1x4 (each wave 128 rows x 32 columns: its B split not shared)
mkdir -p gpurun_out
MSL_H3_W14=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread \
  -k "f16x3 and (dconv or pconv or aspp or kat or accurate or hybrid or residual)" > gpurun_out/w14_tests.log 2>&1 || { tail -40 gpurun_out/w14_tests.log; exit 1; }
tail -2 gpurun_out/w14_tests.log
for v in 0 1 0 1; do
  MSL_H3_W14=$v timeout -k 10 200 python -u scripts/bench_forms.py f16x3 > gpurun_out/w14_$v.jsonl 2>&1 || { tail -20 gpurun_out/w14_$v.jsonl; exit 1; }
  echo "== w14 $v: $(grep '"op"' gpurun_out/w14_$v.jsonl | tail -5 | python3 -c "import sys,json
print(' | '.join(json.loads(l)['op'] + ' ' + str(json.loads(l)['fwd_us']) + '/' + str(json.loads(l)['dgrad_us']) for l in sys.stdin))")"
done
for v in 0 1 0 1; do
  MSL_H3_W14=$v timeout -k 10 300 python -u bench.py --cpu-baseline-iters 0 > gpurun_out/w14_bench_$v.json 2>&1 || { tail -20 gpurun_out/w14_bench_$v.json; exit 1; }
  echo "bench w14 $v $(tail -1 gpurun_out/w14_bench_$v.json | cut -c150-200)"
done
