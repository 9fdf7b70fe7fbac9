#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash gpurun_steps.sh \
  "ESP_GEMM_BM256=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_kernels.py -x -q -k 'bf16 or planes' --timeout 170 --timeout-method thread > gpurun_out/pytest_bm256.log 2>&1" \
  "timeout -k 10 300 python -u bench.py --config c5 --batch 64 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/c5_bm0.log 2>&1" \
  "ESP_GEMM_BM256=1 timeout -k 10 300 python -u bench.py --config c5 --batch 64 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/c5_bm1.log 2>&1" \
  "ESP_GEMM_BM256=1 timeout -k 10 200 python3 tools/gemm_profile.py --batch 64 --config c5 > gpurun_out/gemm_shapes_c5_bm256.txt 2>&1"
