#!/bin/bash
# Run GPU steps in sequence; continue past ordinary test failures (exit 1) but stop at
# anything that looks like a fault / abort / timeout (exit >= 2).
mkdir -p gpurun_out
i=0
for cmd in "$@"; do
  i=$((i+1))
  echo "=== step $i: $cmd" >> gpurun_out/steps.log
  bash -c "$cmd"
  rc=$?
  echo "=== step $i rc=$rc" >> gpurun_out/steps.log
  if [ $rc -ge 2 ]; then echo "stopping after rc=$rc"; exit $rc; fi
done
exit 0
