#!/bin/bash
# round 5: split-K up to 128 splits (d x d weight gradients at two blocks per CU); conv2 forward tile width A/B
# (VARIANT=_c128); per-kernel times
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/prof_f gpurun_out/prof_f128
bash gpurun_steps.sh \
  "timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -k 'gemm or splitk or conv2' -v --maxfail 10 --timeout 350 --timeout-method thread > gpurun_out/r05f_pytest.log 2>&1; rc=\$?; [ \$rc -le 1 ]" \
  "timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/r05f_bench.log 2>&1" \
  "ESP_LIB_VARIANT=_c128 timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/r05f_bench_c128.log 2>&1" \
  "timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/r05f_bench2.log 2>&1" \
  "ESP_LIB_VARIANT=_c128 timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/r05f_bench_c128_2.log 2>&1" \
  "timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_f -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_f.log 2>&1" \
  "ESP_LIB_VARIANT=_c128 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_f128 -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_f128.log 2>&1"
