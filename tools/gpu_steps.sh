#!/bin/bash
# Helper for gpurun calls: run steps in order; a fault/abort/timeout ends the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1  # step logs grow while a step runs
step() {  # step <name> <timeout-seconds> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc" | tee -a gpurun_out/steps.txt
  case $rc in 124|134|137|139|-6|-11) echo "fatal rc $rc in $name: stopping"; exit $rc;; esac
  return $rc
}
