#!/bin/bash
# Split-once GEMM body (ESP_GEMM_X6S=1): prototype numbers, GEMM tests on it, per-shape rates,
# alternating bench runs against the in-register split.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -f gpurun_out/ab.log
bash gpurun_steps.sh \
 "timeout -k 10 200 python tools/x6_proto_bench.py > gpurun_out/x6p2.log 2>&1" \
 "ESP_GEMM_X6S=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k gemm -m gpu -q -x --timeout 150 --timeout-method thread > gpurun_out/pytest_x6s.log 2>&1" \
 "ESP_GEMM_X6S=1 timeout -k 10 200 python tools/gemm_profile.py --batch 128 > gpurun_out/gemm_shapes_x6s.log 2>&1" \
 "bash tools/ab_bench.sh ESP_GEMM_X6S=1 - 2"
