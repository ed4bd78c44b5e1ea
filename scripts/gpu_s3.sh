set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 100 ./scripts/tune_dconv fsk > gpurun_out/tune3.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_s3.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-baseline-iters 0 > gpurun_out/bench_s3.log 2>&1
