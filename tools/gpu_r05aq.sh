#!/bin/bash
# round 5: the conv2 input-gradient class GEMMs on 256 x 128 tiles of 8 waves (diagnostic build _dw) vs default:
# conv2 parity under it, kernel traces
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/prof_aq gpurun_out/prof_aqw
bash gpurun_steps.sh \
  "ESP_LIB_VARIANT=_dw timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_blocks.py tests/test_gpu_fullsize.py -k 'conv2 or subsampl or fullsize_c2' -x -q --timeout 300 --timeout-method thread > gpurun_out/r05aq_pytest_dw.log 2>&1" \
  "timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_aq -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --feed-steps 0 > gpurun_out/prof_aq.log 2>&1" \
  "ESP_LIB_VARIANT=_dw timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_aqw -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --feed-steps 0 > gpurun_out/prof_aqw.log 2>&1"
