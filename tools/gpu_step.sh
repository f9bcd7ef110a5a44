#!/bin/bash
# Run GPU steps in order; stop at the first crash / timeout / fault.
# usage: tools/gpu_step.sh "<timeout_s> <log> <cmd...>" ...
# exit status 1 (ordinary test failures) does not stop the chain.
mkdir -p gpurun_out
for spec in "$@"; do
  t=$(echo "$spec" | awk '{print $1}')
  log=$(echo "$spec" | awk '{print $2}')
  cmd=$(echo "$spec" | cut -d' ' -f3-)
  echo "=== [$t s] $cmd  -> $log"
  start=$(date +%s)
  timeout -k 10 "$t" bash -c "$cmd" > "gpurun_out/$log" 2>&1
  rc=$?
  echo "    rc=$rc  ($(( $(date +%s) - start )) s)"
  tail -n 4 "gpurun_out/$log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "STOP: step failed with rc=$rc"; exit $rc
  fi
done
exit 0
