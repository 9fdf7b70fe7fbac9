#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash gpurun_steps.sh \
  "timeout -k 10 300 python -u -m pytest tests/test_gpu_blocks.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_attn.log 2>&1" \
  "timeout -k 10 120 python -u tools/attn_kernels_bench.py 128 --only probs > gpurun_out/attn_f32.log 2>&1" \
  "ESP_ATTN_XS=1 timeout -k 10 120 python -u tools/attn_kernels_bench.py 128 --only probs > gpurun_out/attn_xs.log 2>&1" \
  "ESP_ATTN_ABL=1 timeout -k 10 120 python -u tools/attn_kernels_bench.py 128 --only probs > gpurun_out/attn_abl_f32.log 2>&1" \
  "timeout -k 10 120 python -u tools/attn_kernels_bench.py 128 --only probs --legacy > gpurun_out/attn_f32_leg.log 2>&1"
