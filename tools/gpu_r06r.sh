#!/bin/bash
# round 6 (r): records at the new default batch (B=384): the default bench line (cpu_baseline leg included),
# a C2 B=384 kernel trace, GEMM-family HBM traffic at B=384 (two --pmc passes)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/prof_r
bash gpurun_steps.sh \
  "timeout -k 10 600 python -u bench.py > gpurun_out/r06r_bench.log 2>&1" \
  "timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --feed-steps 0 > gpurun_out/prof_r.log 2>&1" \
  "TAG=b384 META='384 C2 256,12,0' bash tools/pmc_traffic.sh > gpurun_out/pmc_c2_b384.log 2>&1"
