#!/bin/bash
# bench variants: legacy rel-pos (SLURP YAML default), implicit conv2 input gradient, C4 / C5 lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash gpurun_steps.sh \
  "timeout -k 10 300 python -u bench.py --rel-pos legacy --no-cpu-baseline > gpurun_out/bench_legacy.log 2>&1" \
  "ESP_CONV2_IMPLICIT_DGRAD=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_implicit.log 2>&1" \
  "timeout -k 10 300 python -u bench.py --config c5 --batch 32 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_c5.log 2>&1" \
  "timeout -k 10 300 python -u bench.py --config c4 --batch 32 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_c4.log 2>&1"
