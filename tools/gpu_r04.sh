#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash gpurun_steps.sh \
  "timeout -k 10 600 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_fullsize.py tests/test_gpu_blocks.py tests/test_gpu_model.py -v -x --timeout 170 --timeout-method thread > gpurun_out/pytest_amp.log 2>&1" \
  "timeout -k 10 300 python -u bench.py --config c5 --batch 64 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/c5_attn1.log 2>&1" \
  "timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/c2_head.log 2>&1"
