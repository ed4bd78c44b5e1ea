#!/bin/bash
# f16x3 3x3: shifted B rows as dwordx4 DMAs + read-time border masks. Tests, op timing, bench
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread \
  -k "f16x3" > gpurun_out/bx4_tests.log 2>&1 || { tail -40 gpurun_out/bx4_tests.log; exit 1; }
tail -2 gpurun_out/bx4_tests.log
timeout -k 10 200 python -u scripts/bench_forms.py f16x3 > gpurun_out/bx4_forms.jsonl 2>&1 || { tail -20 gpurun_out/bx4_forms.jsonl; exit 1; }
grep '"op"' gpurun_out/bx4_forms.jsonl | python3 -c "import sys,json
for l in sys.stdin:
  d=json.loads(l); print(d['op'], 'fwd', d['fwd_us'], 'dgrad', d['dgrad_us'], 'wgrad', d['wgrad_us'])"
timeout -k 10 300 python -u bench.py --cpu-baseline-iters 0 > gpurun_out/bx4_bench.json 2>&1 || { tail -20 gpurun_out/bx4_bench.json; exit 1; }
tail -1 gpurun_out/bx4_bench.json | cut -c150-240
python3 -c "import json;d=json.loads(open('gpurun_out/bx4_bench.json').read().strip().split(chr(10))[-1]);print(d['roofline']['kernel_ms'], d['roofline']['frac'])"
