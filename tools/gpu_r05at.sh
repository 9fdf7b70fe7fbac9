#!/bin/bash
# round 5: the FFN w_1 forward on 256 x 128 tiles (default build) vs 128 x 128 (libespnet_mi355_nsw.so): parity, traces
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/prof_at gpurun_out/prof_atn
bash gpurun_steps.sh \
  "timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_blocks.py tests/test_gpu_fullsize.py tests/test_gpu_bench_shape.py tests/test_gpu_model.py -q --timeout 300 --timeout-method thread > gpurun_out/r05at_pytest.log 2>&1" \
  "timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_at -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --feed-steps 0 > gpurun_out/prof_at.log 2>&1" \
  "ESP_LIB_VARIANT=_nsw timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_atn -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --feed-steps 0 > gpurun_out/prof_atn.log 2>&1"
