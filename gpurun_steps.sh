#!/bin/bash
# Runs each argument as one GPU step (each already wrapped in its own `timeout -k`), in order,
# and stops at the first step that fails, times out or faults: no GPU work after a failure.
# usage: bash gpurun_steps.sh "<step 1>" "<step 2>" ...
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
i=0
for step in "$@"; do
  i=$((i + 1))
  echo "[step $i] $step"
  bash -o pipefail -c "$step"
  rc=$?
  echo "[step $i] exit $rc"
  if [ $rc -ne 0 ]; then
    exit $rc
  fi
done
