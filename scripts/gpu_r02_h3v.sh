#!/bin/bash
# f16x3 forward-kernel variants (K-steps per stage, ring depth) on one box, then eager vs graphed bench
mkdir -p gpurun_out
for v in 1,4 1,3 1,5 2,2 1,6 2,3 1,4; do
  echo "== MSL_H3_FWD=$v"
  MSL_H3_FWD=$v timeout -k 10 200 python -u scripts/bench_forms.py f16x3 > gpurun_out/h3v_$v.jsonl 2>&1 || { tail -20 gpurun_out/h3v_$v.jsonl; exit 1; }
  grep '"op"' gpurun_out/h3v_$v.jsonl | tail -5 | python3 -c "import sys,json
for l in sys.stdin:
  d=json.loads(l); print(d['op'], 'fwd', d['fwd_us'], 'dgrad', d['dgrad_us'])"
done
timeout -k 10 300 python -u bench.py --cpu-baseline-iters 0 --graph 0 > gpurun_out/h3v_eager.json 2>&1 || { tail -20 gpurun_out/h3v_eager.json; exit 1; }
tail -1 gpurun_out/h3v_eager.json | cut -c1-260
timeout -k 10 300 python -u bench.py --cpu-baseline-iters 0 > gpurun_out/h3v_graph.json 2>&1 || { tail -20 gpurun_out/h3v_graph.json; exit 1; }
tail -1 gpurun_out/h3v_graph.json | cut -c1-260
