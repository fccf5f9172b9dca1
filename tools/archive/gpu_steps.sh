#!/usr/bin/env bash
# Run GPU steps in order; each under its own time limit.  A step that ends in
# a fault/abort/timeout (exit status other than 0 or 1) stops the script: no
# further GPU work is started in the same call.
#   usage: tools/gpu_steps.sh "<secs>|<name>|<command>" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
status=0
for spec in "$@"; do
  secs=${spec%%|*}; rest=${spec#*|}; name=${rest%%|*}; cmd=${rest#*|}
  echo "=== [$name] ($secs s): $cmd" | tee -a gpurun_out/steps.log
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc in $(( $(date +%s) - start )) s" | tee -a gpurun_out/steps.log
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then
    status=$rc
    if [ $rc -ne 1 ]; then
      echo "=== stopping: step $name ended with rc=$rc" | tee -a gpurun_out/steps.log
      exit $rc
    fi
  fi
done
exit $status
