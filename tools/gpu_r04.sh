#!/bin/bash
# round 4 GPU step list (edited per experiment)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash gpurun_steps.sh \
  "timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py -v -x --timeout 170 --timeout-method thread > gpurun_out/pytest_full.log 2>&1"
