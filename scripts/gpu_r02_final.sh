#!/bin/bash
# Round-2 evidence: full GPU tests + smoke, the dominant op's kernel-trace and PMC passes
# (regenerates profiles' pmc_traffic.json input), bench lines (graph default, eager), and a
# kernel-trace profile of the bench.  usage: scripts/gpu_r02_final.sh <tag>
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
TAG=${1:-r02}
cd $R
./scripts/gpu_steps.sh \
  "900|gpu_tests_$TAG.log|python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu" \
  "200|smoke_$TAG.log|python -c 'import __graft_entry__ as g; g.smoke()'" || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/dom_$TAG -o dom --output-format csv -- python3 $R/scripts/prof_dominant.py 50 > $O/dom_$TAG.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/pmcf_$TAG -o pmcf --output-format csv -- python3 $R/scripts/prof_dominant.py 20 > $O/pmcf_$TAG.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/pmcw_$TAG -o pmcw --output-format csv -- python3 $R/scripts/prof_dominant.py 20 > $O/pmcw_$TAG.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES GRBM_GUI_ACTIVE -d $O/pmcs_$TAG -o pmcs --output-format csv -- python3 $R/scripts/prof_dominant.py 20 > $O/pmcs_$TAG.log 2>&1 || exit $?
python3 $R/scripts/pmc_traffic.py $O/pmcf_$TAG/pmcf_counter_collection.csv $O/pmcw_$TAG/pmcw_counter_collection.csv k_igemm_fwd_sk,k_sk_reduce $O/pmc_traffic_$TAG.json > $O/pmc_$TAG.log 2>&1
cd $R
timeout -k 10 400 python bench.py --pmc $O/pmc_traffic_$TAG.json > $O/bench_$TAG.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --graph 0 --cpu-baseline-iters 0 --pmc $O/pmc_traffic_$TAG.json > $O/bench_eager_$TAG.log 2>&1 || exit $?
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$TAG -o prof --output-format csv -- python3 $R/bench.py --graph 0 --steps 5 --warmup 2 --cpu-baseline-iters 0 > $O/prof_$TAG.log 2>&1
echo done
