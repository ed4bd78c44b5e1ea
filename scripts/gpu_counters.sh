#!/bin/bash
# On the GPU box: hardware counters of one program's kernels, each counter group in a pass of its own
# (rocprofv3 --pmc, no tracing domains besides the kernel trace): HBM traffic (FETCH_SIZE, WRITE_SIZE)
# and two SQ passes (MFMA busy, waits, instruction mix).  Summaries into gpurun_out/<tag>_*.txt.
#   scripts/gpu_counters.sh <tag> <filter[,filter]> <python script> [args...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
TAG=$1; FILT=$2; shift 2
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
run() {  # name, counters...
  local n=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d $O/${TAG}_$n -o $n --output-format csv -- python3 "${PROG[@]}" > $O/${TAG}_$n.log 2>&1
}
PROG=("$@")
run fetch FETCH_SIZE || exit $?
run write WRITE_SIZE || exit $?
run sqa SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_BUSY_CYCLES || exit $?
run sqb SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVES GRBM_GUI_ACTIVE || exit $?
python3 $R/scripts/pmc_traffic.py $O/${TAG}_fetch/fetch_counter_collection.csv $O/${TAG}_write/write_counter_collection.csv $FILT $O/${TAG}_traffic.json ${FORM:-f16x3} > $O/${TAG}_traffic.log 2>&1
python3 $R/scripts/pmc_summary.py $O/${TAG}_sqa/sqa_counter_collection.csv $O/${TAG}_sqb/sqb_counter_collection.csv ${FILT//,/ } > $O/${TAG}_sq.txt 2>&1
