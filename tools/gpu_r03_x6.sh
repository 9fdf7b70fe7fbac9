#!/bin/bash
# fp32 GEMM as bf16x6 split products (experiment build libespnet_mi355_x6.so): accuracy vs fp64
# for both builds, per-shape GEMM rates, A/B bench, then the GPU suite on the experiment build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -f gpurun_out/ab.log
bash gpurun_steps.sh \
 "timeout -k 10 200 python tools/f32_gemm_accuracy.py > gpurun_out/acc_native.log 2>&1" \
 "ESP_LIB_VARIANT=_x6 timeout -k 10 200 python tools/f32_gemm_accuracy.py > gpurun_out/acc_x6.log 2>&1" \
 "ESP_LIB_VARIANT=_x6 timeout -k 10 200 python tools/gemm_profile.py --batch 128 > gpurun_out/gemm_shapes_x6.log 2>&1" \
 "bash tools/ab_bench.sh ESP_LIB_VARIANT=_x6 - 2" \
 "ESP_LIB_VARIANT=_x6 timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread > gpurun_out/pytest_x6.log 2>&1"
