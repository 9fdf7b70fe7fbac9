#!/bin/bash
# round 4 GPU step list (edited per experiment)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash gpurun_steps.sh \
  "timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k 'planes or gemm_f32 or gemm_bf16 or layernorm or bn_swish' --timeout 120 --timeout-method thread > gpurun_out/pytest_pl.log 2>&1" \
  "timeout -k 10 120 python -u -m pytest tests/test_gpu_fullsize.py -x -q -k c4_forward --timeout 120 --timeout-method thread > gpurun_out/pytest_c4f.log 2>&1" \
  "ESP_XPLANES=0 timeout -k 10 120 python -u -m pytest tests/test_gpu_fullsize.py -x -q -k c4_forward --timeout 120 --timeout-method thread > gpurun_out/pytest_c4f_nopl.log 2>&1 || true" \
  "ESP_ATTN_XS=1 timeout -k 10 120 python -u tools/attn_kernels_bench.py 128 --only probs > gpurun_out/attn_xs.log 2>&1" \
  "timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_pl.log 2>&1" \
  "ESP_XPLANES=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_nopl.log 2>&1" \
  "timeout -k 10 300 python -u bench.py --config c5 --batch 64 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_c5.log 2>&1" \
  "ESP_XPLANES=0 timeout -k 10 300 python -u bench.py --config c5 --batch 64 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_c5_nopl.log 2>&1" \
  "timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_bench_shape.py tests/test_gpu_model.py tests/test_gpu_distributed.py -q --timeout 300 --timeout-method thread > gpurun_out/pytest_pl_model.log 2>&1"
