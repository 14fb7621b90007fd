#!/bin/bash
# GPU-box driver: runs named steps, each under its own timeout; stops at the first
# GPU fault / abort / segfault / timeout (exit 124, 134, 137, 139), continues after
# ordinary failures.  Output under gpurun_out/.
#   tools/gpu_run.sh "name:seconds:command" ...
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONDONTWRITEBYTECODE=1
for spec in "$@"; do
  name=${spec%%:*}; rest=${spec#*:}; secs=${rest%%:*}; cmd=${rest#*:}
  echo "=== $name ($secs s): $cmd" | tee -a gpurun_out/steps.log
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc $(( $(date +%s) - start ))s" | tee -a gpurun_out/steps.log
  tail -5 "gpurun_out/$name.log"
  case $rc in 124|134|137|139) echo "fatal rc=$rc: stopping"; exit $rc;; esac
done
exit 0
