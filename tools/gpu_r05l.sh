#!/bin/bash
# round 5: banded dq_v GEMM (esp_relpos_dqv) parity + GEMM MFMA issue order A/B (ESP_LIB_VARIANT=_mo:
# product-major six-product order) + kernel summary
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/prof_l
bash gpurun_steps.sh \
  "timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py -k relpos_dqv -x -v -s --timeout 120 --timeout-method thread > gpurun_out/r05l_pytest0.log 2>&1" \
  "timeout -k 10 700 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_bench_shape.py tests/test_gpu_fullsize.py tests/test_gpu_blocks.py -v -s --maxfail 10 --timeout 350 --timeout-method thread > gpurun_out/r05l_pytest.log 2>&1" \
  "timeout -k 10 400 python -u bench.py --no-cpu-baseline --feed-steps 0 > gpurun_out/r05l_bench.log 2>&1" \
  "ESP_LIB_VARIANT=_mo timeout -k 10 400 python -u bench.py --no-cpu-baseline --feed-steps 0 > gpurun_out/r05l_bench_mo.log 2>&1" \
  "timeout -k 10 400 python -u bench.py --no-cpu-baseline --feed-steps 0 > gpurun_out/r05l_bench2.log 2>&1" \
  "ESP_LIB_VARIANT=_mo timeout -k 10 400 python -u bench.py --no-cpu-baseline --feed-steps 0 > gpurun_out/r05l_bench_mo2.log 2>&1" \
  "timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_l -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --feed-steps 0 > gpurun_out/prof_l.log 2>&1"
