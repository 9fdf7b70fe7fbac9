#!/bin/bash
# round 5 records at HEAD (2): GEMM-family HBM traffic (C2 B=256, C5 B=64), the C5 bench and its kernel summary
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/prof_ao5
bash tools/pmc_traffic.sh && \
BENCH_ARGS="--config c5 --batch 64" TAG=c5 META="64 C5 512,12,1" bash tools/pmc_traffic.sh && \
bash gpurun_steps.sh \
  "timeout -k 10 400 python -u bench.py --config c5 --batch 64 --feed-steps 0 > gpurun_out/r05ao_bench_c5.log 2>&1" \
  "timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ao5 -o run -- python3 bench.py --config c5 --batch 64 --steps 5 --warmup 2 --no-cpu-baseline --feed-steps 0 > gpurun_out/prof_ao5.log 2>&1"
