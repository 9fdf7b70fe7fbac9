#!/bin/bash
# Every BASELINE config's bench line at HEAD (one GPU): legacy rel-pos (the SLURP YAML default),
# variable lengths on one bucketed graph, C4 (d=512, 17 blocks), C5 (bf16) at B=32.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash gpurun_steps.sh \
 "timeout -k 10 300 python bench.py --rel-pos legacy --no-cpu-baseline > gpurun_out/bench_legacy.log 2>&1" \
 "timeout -k 10 300 python bench.py --variable-lengths --no-cpu-baseline > gpurun_out/bench_varlen.log 2>&1" \
 "timeout -k 10 300 python bench.py --config c4 --batch 64 --no-cpu-baseline > gpurun_out/bench_c4.log 2>&1" \
 "timeout -k 10 300 python bench.py --config c5 --batch 32 --no-cpu-baseline > gpurun_out/bench_c5_b32.log 2>&1"
