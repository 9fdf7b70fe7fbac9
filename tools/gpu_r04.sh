#!/bin/bash
# round 4 GPU step list (edited per experiment)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash gpurun_steps.sh \
  "timeout -k 10 600 python -u -m pytest -v tests/test_gpu_fullsize.py -k c5_bf16 --timeout 400 --timeout-method thread > gpurun_out/pytest_r04b.log 2>&1"
