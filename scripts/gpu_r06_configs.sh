#!/bin/bash
# On the GPU box (r06): bench lines of the BASELINE configs at N = 1 (2; 4 at 1280x640 IW + multi; 5, SYNTHIA
# 16 classes at 1280x760 on the fp16 path), the two-pass step (--pair 0) and the bf16 math of config 2, then
# the layer3 3x3 op in the three fp32 forms (scripts/bench_ops.py --form).  Logs: gpurun_out/<tag>_*.
#   scripts/gpu_r06_configs.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-cf}
cd $R && mkdir -p gpurun_out
B="timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-baseline-iters 0"
$B > gpurun_out/${TAG}_cfg2.json 2> gpurun_out/${TAG}_cfg2.err || exit $?
$B --target-mode IW_maxsquare --multi True --lambda-target 0.09 --height 640 --width 1280 > gpurun_out/${TAG}_cfg4.json 2> gpurun_out/${TAG}_cfg4.err || exit $?
$B --num-classes 16 --conv-math fp16 --height 760 --width 1280 --target-mode IW_maxsquare --multi True > gpurun_out/${TAG}_cfg5.json 2> gpurun_out/${TAG}_cfg5.err || exit $?
$B --pair 0 > gpurun_out/${TAG}_twopass.json 2> gpurun_out/${TAG}_twopass.err || exit $?
$B --conv-math bf16 > gpurun_out/${TAG}_cfg2_bf16.json 2> gpurun_out/${TAG}_cfg2_bf16.err || exit $?
for f in f16x3 bf16x6 mfma_f32; do
  timeout -k 10 200 python scripts/bench_ops.py --nimg 2 --reps 20 --only "layer3" --form $f >> gpurun_out/${TAG}_forms.log 2>&1 || exit $?
done
