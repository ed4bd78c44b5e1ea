# Bench lines for BASELINE configs 2, 4 and 5 at N=1 (configs 3-5 name 8 GPUs; per-GPU work is the same)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-baseline-iters 0 > gpurun_out/cfg2.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-baseline-iters 0 --target-mode IW_maxsquare --multi True --lambda-target 0.09 --height 640 --width 1280 > gpurun_out/cfg4.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-baseline-iters 0 --num-classes 16 --conv-math fp16 --height 760 --width 1280 --target-mode IW_maxsquare --multi True > gpurun_out/cfg5.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-baseline-iters 0 --conv-math bf16 > gpurun_out/cfg2_bf16.log 2>&1
