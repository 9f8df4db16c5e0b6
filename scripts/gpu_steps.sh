#!/bin/bash
# Run GPU steps in order; each step under its own time limit.  A plain test failure (rc 1) lets
# the next step run; any crash / abort / timeout code (anything else non-zero) stops the script.
# usage: scripts/gpu_steps.sh "<name>|<seconds>|<command>" ...
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%|*}"; rest="${spec#*|}"; secs="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== [$name] (limit ${secs}s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc"
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
done
exit 0
