#!/bin/bash
# round 6 (p): full GPU suite + smoke at the final HEAD (after the use_amp scaler state)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash gpurun_steps.sh \
  "timeout -k 10 1100 python -u -m pytest tests -m gpu -v -s -rf --timeout 350 --timeout-method thread > gpurun_out/r06p_pytest_gpu.log 2>&1" \
  "timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/r06p_smoke.log 2>&1"
