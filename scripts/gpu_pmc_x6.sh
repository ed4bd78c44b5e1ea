#!/bin/bash
# SQ counters of the bench's dominant op (library default form) in two separate --pmc passes.
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_BUSY_CYCLES \
  -d $O/sq1 -o sq1 --output-format csv -- python3 $R/scripts/prof_dominant.py 20 > $O/sq1.log 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVES GRBM_GUI_ACTIVE \
  -d $O/sq2 -o sq2 --output-format csv -- python3 $R/scripts/prof_dominant.py 20 > $O/sq2.log 2>&1
