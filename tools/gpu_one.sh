#!/bin/bash
# one-off GPU step list (edited per experiment): split-K occupancy target A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash gpurun_steps.sh \
  "ESP_SPLITK_OCC=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_occ.log 2>&1" \
  "timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_occ0.log 2>&1" \
  "ESP_SPLITK_OCC=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_occ1.log 2>&1" \
  "timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_occ0b.log 2>&1" \
  "ESP_SPLITK_OCC=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_occ1b.log 2>&1"
