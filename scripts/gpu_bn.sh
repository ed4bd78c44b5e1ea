set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k bn_act -x -v --timeout 120 --timeout-method thread > gpurun_out/bn_tests.log 2>&1 && \
timeout -k 10 200 python -u scripts/bn_bench.py > gpurun_out/bn_bench.log 2>&1 && \
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_bn.log 2>&1 && \
timeout -k 10 300 python bench.py --cpu-baseline-iters 0 > gpurun_out/bench_bn.log 2>&1
