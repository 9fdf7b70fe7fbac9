#!/bin/bash
# round 5: C2 batch sweep at HEAD, repeated (B per GPU 256 / 384, alternating; B=512 runs out of HBM: 151 GB of graph pool + the eager warm-up)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash gpurun_steps.sh \
  "timeout -k 10 400 python -u bench.py --no-cpu-baseline --feed-steps 0 --steps 10 > gpurun_out/r05v_bench_b256.log 2>&1" \
  "timeout -k 10 400 python -u bench.py --no-cpu-baseline --feed-steps 0 --steps 10 --batch 384 > gpurun_out/r05v_bench_b384.log 2>&1" \
  "timeout -k 10 400 python -u bench.py --no-cpu-baseline --feed-steps 0 --steps 10 > gpurun_out/r05v_bench_b256b.log 2>&1" \
  "timeout -k 10 400 python -u bench.py --no-cpu-baseline --feed-steps 0 --steps 10 --batch 384 > gpurun_out/r05v_bench_b384b.log 2>&1"
