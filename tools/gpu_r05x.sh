#!/bin/bash
# round 5: bf16-operand GEMMs (PREC 2) on 256 x 128 tiles of 8 waves (ESP_GEMM_WIDE=1 ESP_GEMM_WIDE_F32=0,
# libespnet_mi355_wb.so) vs 128 x 128 / 4 waves: bf16 parity under the variant, C5 bench A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash gpurun_steps.sh \
  "ESP_LIB_VARIANT=_wb timeout -k 10 500 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_kernels.py -k 'c5 or bf16 or amp' -x -q --timeout 300 --timeout-method thread > gpurun_out/r05x_pytest_wb.log 2>&1" \
  "timeout -k 10 400 python -u bench.py --config c5 --batch 64 --no-cpu-baseline --feed-steps 0 > gpurun_out/r05x_bench_c5.log 2>&1" \
  "ESP_LIB_VARIANT=_wb timeout -k 10 400 python -u bench.py --config c5 --batch 64 --no-cpu-baseline --feed-steps 0 > gpurun_out/r05x_bench_c5_wb.log 2>&1" \
  "timeout -k 10 400 python -u bench.py --config c5 --batch 64 --no-cpu-baseline --feed-steps 0 > gpurun_out/r05x_bench_c5b.log 2>&1" \
  "ESP_LIB_VARIANT=_wb timeout -k 10 400 python -u bench.py --config c5 --batch 64 --no-cpu-baseline --feed-steps 0 > gpurun_out/r05x_bench_c5_wbb.log 2>&1"
