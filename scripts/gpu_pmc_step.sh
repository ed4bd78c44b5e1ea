#!/bin/bash
# Counters of every kernel of the UDA step (bench.py, eager, 2 timed steps): one SQ/GRBM pass with
# the kernel trace, then FETCH_SIZE and WRITE_SIZE in passes of their own.
# usage: scripts/gpu_pmc_step.sh <tag>
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
TAG=${1:-r02}
B="$R/bench.py --graph 0 --steps 2 --warmup 1 --cpu-baseline-iters 0"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES GRBM_GUI_ACTIVE \
  -d $O/pmcs_${TAG}_sq -o sq --output-format csv -- python3 $B > $O/pmcs_${TAG}_sq.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/pmcs_${TAG}_f -o f --output-format csv -- python3 $B > $O/pmcs_${TAG}_f.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/pmcs_${TAG}_w -o w --output-format csv -- python3 $B > $O/pmcs_${TAG}_w.log 2>&1 || exit $?
echo done
