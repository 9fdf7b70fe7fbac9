#!/bin/bash
# (the ESP_CONV1_FOLD environment switch this ran with is now kernels.CONV1_FOLD: tools/bench_with.py kernels.CONV1_FOLD=0)
# round 6 (i): conv1's weight gradient folded into the conv2 input gradient (esp_conv2_dgrad_c1fold) -- its
# kernel parity test, then the full GPU suite, a C2 B=256 kernel trace with the fold on and off
# (ESP_CONV1_FOLD=0), bench lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/prof_i gpurun_out/prof_i_off
bash gpurun_steps.sh \
  "timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -v -rf -k 'conv' --timeout 120 --timeout-method thread > gpurun_out/r06i_pytest_conv.log 2>&1" \
  "timeout -k 10 1100 python -u -m pytest tests -m gpu -v -s -rf --timeout 350 --timeout-method thread > gpurun_out/r06i_pytest_gpu.log 2>&1" \
  "timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_i -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --feed-steps 0 > gpurun_out/prof_i.log 2>&1" \
  "ESP_CONV1_FOLD=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_i_off -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --feed-steps 0 > gpurun_out/prof_i_off.log 2>&1" \
  "timeout -k 10 300 python -u bench.py --no-cpu-baseline --feed-steps 0 --steps 20 > gpurun_out/r06i_bench.log 2>&1" \
  "ESP_CONV1_FOLD=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline --feed-steps 0 --steps 20 > gpurun_out/r06i_bench_off.log 2>&1"
