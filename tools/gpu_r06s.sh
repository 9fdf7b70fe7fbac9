#!/bin/bash
# round 6 (s): HEAD records of the other configs at the default batch / their batch: legacy C2 (B=384),
# C5 (bf16, B=64), C4 (d=512, 17 blocks, B=64)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash gpurun_steps.sh \
  "timeout -k 10 400 python -u bench.py --rel-pos legacy --no-cpu-baseline --feed-steps 0 > gpurun_out/r06s_bench_legacy_b384.log 2>&1" \
  "timeout -k 10 400 python -u bench.py --config c5 --batch 64 --no-cpu-baseline --feed-steps 0 > gpurun_out/r06s_bench_c5_b64.log 2>&1" \
  "timeout -k 10 400 python -u bench.py --config c4 --batch 64 --no-cpu-baseline --feed-steps 0 > gpurun_out/r06s_bench_c4_b64.log 2>&1"
