#!/bin/bash
# chunked split-K weight gradient: the resident-slot target of the chunk planner (256 / 512 / 1024)
mkdir -p gpurun_out
for v in 512 256 1024 512 256; do
  MSL_WX6_SLOTS=$v timeout -k 10 200 python -u scripts/bench_forms.py f16x3 > gpurun_out/slots_$v.jsonl 2>&1 || { tail -20 gpurun_out/slots_$v.jsonl; exit 1; }
  echo "== slots $v: $(grep '"op"' gpurun_out/slots_$v.jsonl | tail -5 | python3 -c "import sys,json
print(' '.join(json.loads(l)['op'] + ' ' + str(json.loads(l)['wgrad_us']) for l in sys.stdin))")"
done
for v in 512 256; do
  MSL_WX6_SLOTS=$v timeout -k 10 300 python -u bench.py --cpu-baseline-iters 0 > gpurun_out/slots_bench_$v.json 2>&1 || { tail -20 gpurun_out/slots_bench_$v.json; exit 1; }
  echo "bench slots $v $(tail -1 gpurun_out/slots_bench_$v.json | cut -c150-200)"
done
