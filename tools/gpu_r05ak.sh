#!/bin/bash
# round 5: legacy length-bucketed batches under the opt-in flash / score-gradient attention forms
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash gpurun_steps.sh \
  "timeout -k 10 600 python -u -m pytest tests/test_gpu_buckets.py tests/test_gpu_flash.py -v --timeout 300 --timeout-method thread > gpurun_out/r05ak_pytest_buckets.log 2>&1"
