#!/bin/bash
# Run GPU steps in order, each under its own time limit.  An ordinary failure (exit 1/2) is
# logged and the next step runs; a crash, abort or timeout (124/134/137/139) ends the call.
# usage: tools/gpu_steps.sh "name:seconds:command" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; secs="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== $name (limit ${secs}s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc ($(( $(date +%s) - start ))s)"
  tail -n 25 "gpurun_out/$name.log"
  case $rc in
    124|134|137|139) echo "STOP: $name crashed or timed out"; exit $rc ;;
  esac
done
exit 0
