#!/bin/bash
# round 5: GEMM tile-width near-ties -> 128 (VARIANT=_t128, ESP_GEMM_TILE_TIE=0.95) vs default; C2 and C5
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/prof_g gpurun_out/prof_gt
bash gpurun_steps.sh \
  "timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/r05g_bench.log 2>&1" \
  "ESP_LIB_VARIANT=_t128 timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/r05g_bench_t.log 2>&1" \
  "timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/r05g_bench2.log 2>&1" \
  "ESP_LIB_VARIANT=_t128 timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/r05g_bench_t2.log 2>&1" \
  "timeout -k 10 400 python -u bench.py --config c5 --batch 64 --no-cpu-baseline > gpurun_out/r05g_c5.log 2>&1" \
  "ESP_LIB_VARIANT=_t128 timeout -k 10 400 python -u bench.py --config c5 --batch 64 --no-cpu-baseline > gpurun_out/r05g_c5_t.log 2>&1" \
  "timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_g -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_g.log 2>&1" \
  "ESP_LIB_VARIANT=_t128 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_gt -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_gt.log 2>&1"
