#!/bin/bash
# Run GPU steps in order, each under its own time limit. Test failures (rc 1) continue;
# any other non-zero status (fault, abort, timeout) ends the script: nothing more on the GPU.
# usage: tools/gpu_steps.sh "<secs>|<name>|<command>" ...
mkdir -p gpurun_out
for spec in "$@"; do
  secs="${spec%%|*}"; rest="${spec#*|}"; name="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== [$name] $cmd (limit ${secs}s)"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc in $(( $(date +%s) - start ))s"
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "=== stopping after rc=$rc"; exit $rc; fi
done
