#!/bin/bash
# attention kernel iteration: block tests + microbench (key-split and single-wave forms)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash gpurun_steps.sh \
  "timeout -k 10 300 python -u -m pytest tests/test_gpu_blocks.py tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread > gpurun_out/blocks.log 2>&1" \
  "timeout -k 10 120 python -u tools/attn_bench.py 128 --fwd-only > gpurun_out/attn_bench.log 2>&1" \
  "ESP_ATTN_SPLIT=1 timeout -k 10 120 python -u tools/attn_bench.py 128 --fwd-only > gpurun_out/attn_bench_split1.log 2>&1"
