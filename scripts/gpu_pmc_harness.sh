#!/bin/bash
# SQ / GRBM counters of the tuning harness's kernels (two --pmc passes, kernel trace only).
# usage: scripts/gpu_pmc_harness.sh <harness mode> <tag>
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
MODE=$1; TAG=$2
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_BUSY_CYCLES \
  -d $O/pmc_${TAG}_1 -o p1 --output-format csv -- $R/scripts/tune_dconv $MODE > $O/pmc_${TAG}_1.log 2>&1
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVES GRBM_GUI_ACTIVE \
  -d $O/pmc_${TAG}_2 -o p2 --output-format csv -- $R/scripts/tune_dconv $MODE > $O/pmc_${TAG}_2.log 2>&1
echo done
