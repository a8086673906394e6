#!/bin/bash
# Run GPU steps in order; stop at the first fault/abort/timeout (never retry).
# usage: bash bench/gpu_steps.sh "<name>:<timeout>:<cmd>" ...
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONPATH="$GRAFT_REPO_ROOT" LZK_AUTOBUILD=0
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; to="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== $name (timeout ${to}s): $cmd" | tee -a gpurun_out/steps.log
  timeout -k 10 "$to" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/steps.log
  tail -5 "gpurun_out/$name.log"
  case $rc in
    0|1|2|5) ;;            # ok / test failures: keep going
    *) echo "fatal rc=$rc, stopping"; exit $rc ;;
  esac
done
