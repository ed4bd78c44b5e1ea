#!/bin/bash
# Run GPU steps in order: "seconds|logname|command" per argument.  Each step has its own time
# limit; a step that times out, aborts or crashes (rc 124/134/137/139 or > 128) ends the batch,
# an ordinary failure (a failing test) does not.
mkdir -p gpurun_out
for spec in "$@"; do
  secs="${spec%%|*}"; rest="${spec#*|}"; log="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== $(date +%T) step $log: $cmd" | tee -a gpurun_out/steps.log
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$log" 2>&1
  rc=$?
  echo "=== $(date +%T) step $log rc=$rc" | tee -a gpurun_out/steps.log
  tail -3 "gpurun_out/$log"
  if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then echo "fatal rc $rc: stopping"; exit $rc; fi
done
