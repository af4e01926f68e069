#!/bin/bash
# Runs GPU steps in sequence on the gpurun box; each step has its own time
# limit; stops at the first crash/timeout (rc not in {0,1}) so nothing more
# touches the GPU after a fault.  Usage: tools/gpu_steps.sh "<secs>:<name>:<cmd>" ...
export TMPDIR=/tmp
mkdir -p gpurun_out
for spec in "$@"; do
  secs="${spec%%:*}"; rest="${spec#*:}"; name="${rest%%:*}"; cmd="${rest#*:}"
  echo "== step $name (limit ${secs}s): $cmd" >> gpurun_out/steps.log
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "== step $name rc=$rc" >> gpurun_out/steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "stopping after $name (rc=$rc)" >> gpurun_out/steps.log
    exit $rc
  fi
done
exit 0
