#!/bin/bash
# round 5: C5 per-kernel traces, bf16-operand GEMMs on 2-slab 256 x 128 / 8-wave tiles (libespnet_mi355_wb2.so) vs default
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/prof_ap gpurun_out/prof_apw
bash gpurun_steps.sh \
  "ESP_LIB_VARIANT=_wb2 timeout -k 10 500 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_kernels.py -k 'c5 or bf16 or amp' -x -q --timeout 300 --timeout-method thread > gpurun_out/r05ap_pytest_wb2.log 2>&1" \
  "timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ap -o run -- python3 bench.py --config c5 --batch 64 --steps 5 --warmup 2 --no-cpu-baseline --feed-steps 0 > gpurun_out/prof_ap.log 2>&1" \
  "ESP_LIB_VARIANT=_wb2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_apw -o run -- python3 bench.py --config c5 --batch 64 --steps 5 --warmup 2 --no-cpu-baseline --feed-steps 0 > gpurun_out/prof_apw.log 2>&1"
