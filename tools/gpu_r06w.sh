#!/bin/bash
# round 6 (w): final HEAD record after the fold-epilogue change -- full GPU suite, smoke, the default bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash gpurun_steps.sh \
  "timeout -k 10 1100 python -u -m pytest tests -m gpu -v -s -rf --timeout 350 --timeout-method thread > gpurun_out/r06w_pytest_gpu.log 2>&1" \
  "timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/r06w_smoke.log 2>&1" \
  "timeout -k 10 600 python -u bench.py > gpurun_out/r06w_bench.log 2>&1"
