#!/bin/bash
# final r02 tree: full GPU suite, smoke, bench with CPU baseline + PMC file, step kernel trace
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  > gpurun_out/fin_tests.log 2>&1; rc=$?; tail -2 gpurun_out/fin_tests.log; grep -E 'FAILED|ERROR' gpurun_out/fin_tests.log | head
[ $rc -le 1 ] || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin_smoke.log 2>&1 || { tail -20 gpurun_out/fin_smoke.log; exit 1; }
tail -1 gpurun_out/fin_smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/fin_bench.json 2> gpurun_out/fin_bench.err || { tail -30 gpurun_out/fin_bench.err; exit 1; }
cut -c1-330 gpurun_out/fin_bench.json
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fin_prof -o prof --output-format csv -- python3 -u bench.py --steps 10 --warmup 3 \
  --cpu-baseline-iters 0 > gpurun_out/fin_prof_bench.json 2> gpurun_out/fin_prof_bench.err || { tail -30 gpurun_out/fin_prof_bench.err; exit 1; }
cut -c1-200 gpurun_out/fin_prof_bench.json
