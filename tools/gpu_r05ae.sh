#!/bin/bash
# round 5: non-temporal stores of the conv2 input gradient output (ESP_CONV2_DGRAD_NT=1, libespnet_mi355_dn.so)
# vs plain: conv2 parity under the variant, kernel traces, benches
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/prof_ae gpurun_out/prof_aen
bash gpurun_steps.sh \
  "ESP_LIB_VARIANT=_dn timeout -k 10 400 python -u -m pytest tests/test_gpu_blocks.py tests/test_gpu_kernels.py tests/test_gpu_fullsize.py -k 'conv or subsampl or fullsize_c2' -q --timeout 300 --timeout-method thread > gpurun_out/r05ae_pytest.log 2>&1" \
  "timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ae -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --feed-steps 0 > gpurun_out/prof_ae.log 2>&1" \
  "ESP_LIB_VARIANT=_dn timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_aen -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --feed-steps 0 > gpurun_out/prof_aen.log 2>&1" \
  "timeout -k 10 400 python -u bench.py --no-cpu-baseline --feed-steps 0 > gpurun_out/r05ae_bench.log 2>&1" \
  "ESP_LIB_VARIANT=_dn timeout -k 10 400 python -u bench.py --no-cpu-baseline --feed-steps 0 > gpurun_out/r05ae_bench_dn.log 2>&1"
