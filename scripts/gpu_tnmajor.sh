#!/bin/bash
# Stream-K tile order A/B: timings (reg2) and FETCH/WRITE of the layer3 x6p op (reg3), both builds.
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
cd $R
./scripts/gpu_steps.sh "150|tn_m.log|./scripts/tune_dconv reg2" "150|tn_n.log|./scripts/tune_dconv_tn reg2" || exit $?
cd /tmp && export TMPDIR=/tmp
for b in tune_dconv tune_dconv_tn; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $c -d $O/pmc_${b}_$c -o p --output-format csv -- $R/scripts/$b reg3 > $O/pmc_${b}_$c.log 2>&1 || exit $?
  done
done
echo done
