set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python bench.py --cpu-baseline-iters 0 > gpurun_out/r4base_bench.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r4base_prof -o prof --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --cpu-baseline-iters 0 > $R/gpurun_out/r4base_prof.log 2>&1
