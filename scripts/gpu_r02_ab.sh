#!/bin/bash
# Same-box A/B of the forward-form schedule: 1x1 dispatch timings with the hybrid schedule on,
# off, on again (box-to-box clocks differ by ~20 % on the x6 kernels), plus the GPU's clocks.
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
TAG=${1:-ab}
(rocm-smi --showclocks --showpower --showtemp > gpurun_out/smi_$TAG.log 2>&1 || true)
./scripts/gpu_steps.sh \
  "300|d1x1_${TAG}_on.log|python -u scripts/bench_conv1x1_dispatch.py --sk-hybrid 1" \
  "300|d1x1_${TAG}_off.log|python -u scripts/bench_conv1x1_dispatch.py --sk-hybrid 0" \
  "300|d1x1_${TAG}_on2.log|python -u scripts/bench_conv1x1_dispatch.py --sk-hybrid 1" || exit $?
(rocm-smi --showclocks --showpower --showtemp >> gpurun_out/smi_$TAG.log 2>&1 || true)
