#!/bin/bash
# round 5: the GPU suite once more at HEAD (after the prologue-barrier fix) and a bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash gpurun_steps.sh \
  "timeout -k 10 1100 python -u -m pytest tests -m gpu -q --timeout 350 --timeout-method thread > gpurun_out/r05as_pytest_gpu.log 2>&1" \
  "timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/r05as_bench.log 2>&1"
