#!/bin/bash
# round 5: block-staged probabilities kernel -- attention / full-size parity, kernel A/B vs the per-wave
# kernel (libespnet_mi355_w.so), C2 bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash gpurun_steps.sh \
  "timeout -k 10 900 python -u -m pytest tests/test_gpu_blocks.py tests/test_gpu_bench_shape.py tests/test_gpu_fullsize.py tests/test_slurp_config.py tests/test_gpu_bf16.py tests/test_gpu_buckets.py -v -s --maxfail 10 --timeout 350 --timeout-method thread > gpurun_out/r05b_pytest.log 2>&1; rc=\$?; [ \$rc -le 1 ]" \
  "for v in '' _w; do for l in '' --legacy; do echo \"variant=\$v \$l\"; ESP_LIB_VARIANT=\$v timeout -k 10 120 python -u tools/attn_kernels_bench.py 256 --only probs \$l || exit 1; done; done > gpurun_out/r05b_attn_ab.txt 2>&1" \
  "timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/r05b_bench.log 2>&1" \
  "ESP_LIB_VARIANT=_w timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/r05b_bench_w.log 2>&1"
