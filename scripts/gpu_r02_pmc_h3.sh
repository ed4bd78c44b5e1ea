#!/bin/bash
# f16x3 counters: the dominant op's SQ/GRBM passes, then every kernel of the step (three passes)
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_BUSY_CYCLES \
  -d $O/h3sq1 -o sq1 --output-format csv -- python3 $R/scripts/prof_dominant.py 20 > $O/h3sq1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVES GRBM_GUI_ACTIVE \
  -d $O/h3sq2 -o sq2 --output-format csv -- python3 $R/scripts/prof_dominant.py 20 > $O/h3sq2.log 2>&1 || exit $?
bash $R/scripts/gpu_pmc_step.sh r02h3 || exit $?
