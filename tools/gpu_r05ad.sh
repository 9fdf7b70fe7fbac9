#!/bin/bash
# round 5: non-temporal stores of P / P_drop in the probabilities kernel (default) vs plain (ESP_ATTN_NT=0,
# libespnet_mi355_an.so), with the conv1 non-temporal stores in both: attention parity, kernel traces, benches
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/prof_ad gpurun_out/prof_adn
bash gpurun_steps.sh \
  "timeout -k 10 400 python -u -m pytest tests/test_gpu_blocks.py tests/test_gpu_kernels.py -k 'attn or relpos or conv1 or subsampl' -q --timeout 300 --timeout-method thread > gpurun_out/r05ad_pytest.log 2>&1" \
  "timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ad -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --feed-steps 0 > gpurun_out/prof_ad.log 2>&1" \
  "ESP_LIB_VARIANT=_an timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_adn -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --feed-steps 0 > gpurun_out/prof_adn.log 2>&1" \
  "timeout -k 10 400 python -u bench.py --no-cpu-baseline --feed-steps 0 > gpurun_out/r05ad_bench.log 2>&1" \
  "ESP_LIB_VARIANT=_an timeout -k 10 400 python -u bench.py --no-cpu-baseline --feed-steps 0 > gpurun_out/r05ad_bench_an.log 2>&1"
