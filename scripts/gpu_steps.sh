#!/bin/bash
# Run GPU steps in order; stop at the first fault/abort/timeout (exit 124,134,137,139 or
# signal), continue past ordinary test failures.  Usage: scripts/gpu_steps.sh name:secs:cmd ...
# A heartbeat file under gpurun_out/ is appended every 50 s while the steps run (long
# benchmark steps print only at their end); it stops with the script.
mkdir -p gpurun_out
( while true; do date +%s >> gpurun_out/heartbeat.log; sleep 50; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; secs="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== $name ($secs s): $cmd" >> gpurun_out/steps.log
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc" >> gpurun_out/steps.log
  tail -3 "gpurun_out/$name.log" >> gpurun_out/steps.log
  case $rc in
    124|134|137|139|143) echo "fatal rc=$rc in $name; stopping" >> gpurun_out/steps.log; exit $rc;;
  esac
done
exit 0
