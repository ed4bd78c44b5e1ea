#!/bin/bash
# same-box A/B of the f16x3 / fp16 forward stage with every LDS read of a K-step issued before
# the B split and product-major MFMA order (new) vs the previous library (_lib/libmsl_hip_base.so)
mkdir -p gpurun_out
L=maxsquareloss_amd/_lib
cp $L/libmsl_hip.so $L/libmsl_hip_new.so
run_ab() {  # $1 = tag
  timeout -k 10 200 python -u scripts/bench_forms.py f16x3 > gpurun_out/ilp_forms_$1.jsonl 2> gpurun_out/ilp_forms_$1.err || { tail -20 gpurun_out/ilp_forms_$1.err; return 1; }
  timeout -k 10 300 python -u bench.py --cpu-baseline-iters 0 > gpurun_out/ilp_bench_$1.json 2> gpurun_out/ilp_bench_$1.err || { tail -20 gpurun_out/ilp_bench_$1.err; return 1; }
  echo "== $1"; cut -c1-200 gpurun_out/ilp_bench_$1.json
}
run_ab new1 && cp $L/libmsl_hip_base.so $L/libmsl_hip.so && run_ab base1 && cp $L/libmsl_hip_new.so $L/libmsl_hip.so && run_ab new2 || exit 1
timeout -k 10 240 python -u bench.py --cpu-baseline-iters 0 --conv-math fp16 > gpurun_out/ilp_bench_fp16_new.json 2>&1 || exit 1
cut -c1-200 gpurun_out/ilp_bench_fp16_new.json | tail -1
