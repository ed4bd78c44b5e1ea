#!/bin/bash
# final tree (LDS reads of a K-step issued ahead of the B split, product-major MFMAs): full GPU
# suite + smoke, the dominant-kernel profile, its PMC traffic, the bench line and a step kernel trace
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  > gpurun_out/fin4_tests.log 2>&1; rc=$?; tail -2 gpurun_out/fin4_tests.log; grep -E 'FAILED|ERROR' gpurun_out/fin4_tests.log | head
[ $rc -le 1 ] || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin4_smoke.log 2>&1 || { tail -20 gpurun_out/fin4_smoke.log; exit 1; }
tail -1 gpurun_out/fin4_smoke.log
bash scripts/gpu_bench_prof.sh r02i f16x3 || exit 1
cat gpurun_out/pmc_r02i.log
tail -1 gpurun_out/bench_r02i.log | cut -c1-300
