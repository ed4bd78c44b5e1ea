#!/bin/bash
# On the GPU box: per-op GEMM timings at the step's pair shapes, the default bench line, then the ASPP
# head profile (scripts/gpu_aspp_prof.sh).  TAG names the outputs.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-ops}
cd $R && mkdir -p gpurun_out
timeout -k 10 200 python scripts/bench_ops.py --nimg 2 --reps 30 > gpurun_out/${TAG}_ops.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --cpu-baseline-iters 0 > gpurun_out/${TAG}_bench.json 2>/dev/null || exit $?
bash scripts/gpu_aspp_prof.sh ${TAG}_aspp
