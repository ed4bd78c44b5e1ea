set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 200 ./scripts/tune_dconv > gpurun_out/tune.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-baseline-iters 0 > gpurun_out/bench_t.log 2>&1
