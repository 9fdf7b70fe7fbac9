#!/bin/bash
# round 4: C5 records at HEAD -- bench, rocprof kernel summary, GEMM-family HBM traffic
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/prof_c5
bash gpurun_steps.sh \
  "timeout -k 10 400 python -u bench.py --config c5 --batch 64 > gpurun_out/bench_c5_head.log 2>&1" \
  "timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5 -o run -- python3 bench.py --config c5 --batch 64 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_c5.log 2>&1" \
  "BENCH_ARGS='--config c5 --batch 64' TAG=c5 META='64 C5 512,12,1' bash tools/pmc_traffic.sh > gpurun_out/pmc_c5.log 2>&1"
