#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash gpurun_steps.sh \
  "timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_fullsize.py tests/test_gpu_bf16.py tests/test_gpu_graph.py tests/test_gpu_trainer.py -x -q --timeout 170 --timeout-method thread > gpurun_out/pytest_flat.log 2>&1" \
  "timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/b_flat1.log 2>&1" \
  "ESP_FLAT_CAST=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/b_flat0.log 2>&1" \
  "timeout -k 10 300 python -u bench.py --config c5 --batch 64 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/b5_flat1.log 2>&1" \
  "ESP_FLAT_CAST=0 timeout -k 10 300 python -u bench.py --config c5 --batch 64 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/b5_flat0.log 2>&1"
