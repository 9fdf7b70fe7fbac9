#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash gpurun_steps.sh \
  "timeout -k 10 200 python3 tools/gemm_profile.py --batch 128 > gpurun_out/gs_default.txt 2>&1" \
  "ESP_CONV2_DGRAD_BNT=64 timeout -k 10 200 python3 tools/gemm_profile.py --batch 128 > gpurun_out/gs_dg64.txt 2>&1" \
  "ESP_SPLITK_TARGET=1024 timeout -k 10 200 python3 tools/gemm_profile.py --batch 128 > gpurun_out/gs_sk1024.txt 2>&1" \
  "ESP_SPLITK_TARGET=256 timeout -k 10 200 python3 tools/gemm_profile.py --batch 128 > gpurun_out/gs_sk256.txt 2>&1"
