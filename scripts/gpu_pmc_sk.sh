#!/bin/bash
# PMC passes over the stream-K conv kernel (run on the GPU box; counters in separate passes).
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_BUSY_CYCLES \
  -d $R/gpurun_out/pmc1 -o pmc1 --output-format csv -- $R/scripts/tune_dconv sk > $R/gpurun_out/pmc1.log 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVES GRBM_GUI_ACTIVE \
  -d $R/gpurun_out/pmc2 -o pmc2 --output-format csv -- $R/scripts/tune_dconv sk > $R/gpurun_out/pmc2.log 2>&1
