#!/bin/bash
# SQ/GRBM counters of the dominant op (layer3 dconv fwd, f16x3) on the current stage schedule
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_BUSY_CYCLES \
  -d $O/sq2a -o sqa --output-format csv -- python3 $R/scripts/prof_dominant.py 20 > $O/sq2a.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVES GRBM_GUI_ACTIVE \
  -d $O/sq2b -o sqb --output-format csv -- python3 $R/scripts/prof_dominant.py 20 > $O/sq2b.log 2>&1 || exit $?
python3 $R/scripts/pmc_summary.py $O/sq2a/sqa_counter_collection.csv $O/sq2b/sqb_counter_collection.csv k_igemm_fwd_sk k_sk_reduce > $O/sq2_dom.txt && cat $O/sq2_dom.txt
