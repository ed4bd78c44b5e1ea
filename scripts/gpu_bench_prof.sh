#!/bin/bash
# On the GPU box: the bench line, a kernel-trace profile of the same bench, a kernel-trace
# profile of the dominant kernel alone, and its PMC HBM traffic (separate --pmc passes).
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-r01}
O=$R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/dom_$TAG -o dom --output-format csv -- python3 $R/scripts/prof_dominant.py 50 > $O/dom_$TAG.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmcf_$TAG -o pmcf --output-format csv -- python3 $R/scripts/prof_dominant.py 20 > $O/pmcf_$TAG.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmcw_$TAG -o pmcw --output-format csv -- python3 $R/scripts/prof_dominant.py 20 > $O/pmcw_$TAG.log 2>&1
python3 $R/scripts/pmc_traffic.py $O/pmcf_$TAG/pmcf_counter_collection.csv $O/pmcw_$TAG/pmcw_counter_collection.csv k_igemm_fwd_sk,k_sk_reduce $O/pmc_traffic_$TAG.json ${2:-f16x3} > $O/pmc_$TAG.log 2>&1
cd $R
timeout -k 10 400 python bench.py --pmc $O/pmc_traffic_$TAG.json > $O/bench_$TAG.log 2>&1
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$TAG -o prof --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --cpu-baseline-iters 0 > $O/prof_$TAG.log 2>&1
