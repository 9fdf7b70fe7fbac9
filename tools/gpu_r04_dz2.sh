#!/bin/bash
# round 4: dz2 written as bf16 by the out-Linear input gradient in the bf16 mode (EPI_RMASK_PL) -- bf16 / C5 /
# kernel / block tests, same-box A/B at C5 B=64 (ESP_DZ2_DIRECT 0 / 1 alternating)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash gpurun_steps.sh \
  "timeout -k 10 600 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_fullsize.py tests/test_gpu_kernels.py tests/test_gpu_blocks.py -m gpu -v --timeout 250 --timeout-method thread > gpurun_out/pytest_dz2.log 2>&1" \
  "ESP_DZ2_DIRECT=0 timeout -k 10 300 python -u bench.py --config c5 --batch 64 --no-cpu-baseline > gpurun_out/ab_dz0a.log 2>&1" \
  "ESP_DZ2_DIRECT=1 timeout -k 10 300 python -u bench.py --config c5 --batch 64 --no-cpu-baseline > gpurun_out/ab_dz1a.log 2>&1" \
  "ESP_DZ2_DIRECT=0 timeout -k 10 300 python -u bench.py --config c5 --batch 64 --no-cpu-baseline > gpurun_out/ab_dz0b.log 2>&1" \
  "ESP_DZ2_DIRECT=1 timeout -k 10 300 python -u bench.py --config c5 --batch 64 --no-cpu-baseline > gpurun_out/ab_dz1b.log 2>&1"
