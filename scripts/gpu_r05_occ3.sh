#!/bin/bash
# On the GPU box (r05): the BD forward at three waves per SIMD (probe build, 768 workers) vs two.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
OUT=gpurun_out/r05_occ3.log
: > $OUT
for shp in "256 256 65 129 2 2" "128 128 65 129 2 1" "512 512 65 129 2 4"; do
  timeout -k 10 120 python scripts/probe_sk.py $shp >> $OUT 2>&1 || exit $?
done
