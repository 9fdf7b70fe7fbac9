#!/bin/bash
# Round-3 A/B: GEMM tests, bench, per-shape GEMM timings with and without 64-row tiles, C5 line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash gpurun_steps.sh \
 "timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_bf16.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gemm.log 2>&1" \
 "timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1" \
 "timeout -k 10 200 python tools/gemm_profile.py --batch 128 > gpurun_out/gemm_shapes.log 2>&1" \
 "ESP_GEMM_NO_BM64=1 timeout -k 10 200 python tools/gemm_profile.py --batch 128 > gpurun_out/gemm_shapes_nobm64.log 2>&1" \
 "ESP_GEMM_NO_BM64=1 timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/bench_nobm64.log 2>&1" \
 "timeout -k 10 300 python bench.py --config c5 --batch 64 --no-cpu-baseline > gpurun_out/bench_c5.log 2>&1"
