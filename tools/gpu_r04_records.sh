#!/bin/bash
# round 4 records at HEAD: C2 bench, rocprof kernel summary (C2, C5), GEMM-family HBM traffic (C2, C5)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/prof gpurun_out/prof_c5
bash gpurun_steps.sh \
  "timeout -k 10 400 python -u bench.py > gpurun_out/bench_head.log 2>&1" \
  "timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof.log 2>&1" \
  "timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5 -o run -- python3 bench.py --config c5 --batch 64 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_c5.log 2>&1" \
  "TAG=c2 bash tools/pmc_traffic.sh > gpurun_out/pmc_c2.log 2>&1" \
  "BENCH_ARGS='--config c5 --batch 64' TAG=c5 META='64 C5 512,12,1' bash tools/pmc_traffic.sh > gpurun_out/pmc_c5.log 2>&1"
