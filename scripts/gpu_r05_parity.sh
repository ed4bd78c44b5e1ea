#!/bin/bash
# On the GPU box (r05): the parity tests this round added or changed (full-size logits, the config-5
# fp16 envelope against the oracle's fp16-operand emulation, the shift form in bf16 / fp16, graph
# replays with the shift packs batched), printed margins (-s), then the default bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-p}
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -s -v --timeout 600 --timeout-method thread -m gpu \
  tests/test_gpu_configs.py tests/test_gpu_graph.py \
  "tests/test_gpu_ops.py::test_aspp_shift_form_low_precision" "tests/test_gpu_ops.py::test_pack_batch_matches_per_conv_packs" \
  > gpurun_out/parity_$TAG.log 2>&1
rc=$?
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
exit $rc
