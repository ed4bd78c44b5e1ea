# kernel-trace profile of the bench and of the BN A/B microbench (per-kernel durations)
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-x}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o prof --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --cpu-baseline-iters 0 > $R/gpurun_out/prof_$TAG.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/profbn_$TAG -o prof --output-format csv -- python3 $R/scripts/bn_bench.py > $R/gpurun_out/profbn_$TAG.log 2>&1
