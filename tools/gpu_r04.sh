#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash gpurun_steps.sh \
  "timeout -k 10 120 python -u tools/attn_kernels_bench.py 128 --only probs > gpurun_out/attn_a0.log 2>&1" \
  "ESP_ATTN_ABL=1 timeout -k 10 120 python -u tools/attn_kernels_bench.py 128 --only probs > gpurun_out/attn_a1.log 2>&1" \
  "ESP_ATTN_ABL=5 timeout -k 10 120 python -u tools/attn_kernels_bench.py 128 --only probs > gpurun_out/attn_a5.log 2>&1" \
  "ESP_ATTN_ABL=4 timeout -k 10 120 python -u tools/attn_kernels_bench.py 128 --only probs > gpurun_out/attn_a4.log 2>&1" \
  "ESP_ATTN_XS=1 ESP_ATTN_ABL=5 timeout -k 10 120 python -u tools/attn_kernels_bench.py 128 --only probs > gpurun_out/attn_a5xs.log 2>&1"
