#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash gpurun_steps.sh \
  "timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -v -x -k 'conv2 or conv1 or bf16' --timeout 120 --timeout-method thread > gpurun_out/pytest_conv.log 2>&1" \
  "timeout -k 10 600 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_fullsize.py tests/test_gpu_blocks.py tests/test_gpu_model.py -x -q --timeout 170 --timeout-method thread > gpurun_out/pytest_amp.log 2>&1" \
  "timeout -k 10 300 python -u bench.py --config c5 --batch 64 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/c5_conv.log 2>&1" \
  "timeout -k 10 200 python3 tools/gemm_profile.py --batch 64 --config c5 > gpurun_out/gemm_shapes_c5_conv.txt 2>&1"
