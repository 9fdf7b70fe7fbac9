#!/bin/bash
# round 4: the whole GPU suite + smoke (round-end records)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash gpurun_steps.sh \
  "timeout -k 10 1500 python -u -m pytest tests -m gpu -v --timeout 170 --timeout-method thread > gpurun_out/pytest_gpu_all.log 2>&1" \
  "timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/smoke.log 2>&1"
