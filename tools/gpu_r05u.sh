#!/bin/bash
# round 5: C2 batch sweep at HEAD (B per GPU 256 / 320 / 384; the headline keeps the fastest that fits)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash gpurun_steps.sh \
  "timeout -k 10 400 python -u bench.py --no-cpu-baseline --feed-steps 0 --steps 10 > gpurun_out/r05u_bench_b256.log 2>&1" \
  "timeout -k 10 400 python -u bench.py --no-cpu-baseline --feed-steps 0 --steps 10 --batch 320 > gpurun_out/r05u_bench_b320.log 2>&1" \
  "timeout -k 10 400 python -u bench.py --no-cpu-baseline --feed-steps 0 --steps 10 --batch 384 > gpurun_out/r05u_bench_b384.log 2>&1"
