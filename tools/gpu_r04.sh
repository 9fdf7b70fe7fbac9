#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash gpurun_steps.sh \
  "timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_blocks.py tests/test_gpu_model.py tests/test_gpu_fullsize.py -x -q --timeout 170 --timeout-method thread > gpurun_out/pytest_fin.log 2>&1" \
  "timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/b_fin.log 2>&1" \
  "timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof.log 2>&1"
