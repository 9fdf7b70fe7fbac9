#!/bin/bash
# round 4: same-box A/B of the planes-path dy memo at C5 B=64 (alternating)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash gpurun_steps.sh \
  "ESP_PLANES_DY_MEMO=0 timeout -k 10 300 python -u bench.py --config c5 --batch 64 --no-cpu-baseline > gpurun_out/ab_memo0a.log 2>&1" \
  "ESP_PLANES_DY_MEMO=1 timeout -k 10 300 python -u bench.py --config c5 --batch 64 --no-cpu-baseline > gpurun_out/ab_memo1a.log 2>&1" \
  "ESP_PLANES_DY_MEMO=0 timeout -k 10 300 python -u bench.py --config c5 --batch 64 --no-cpu-baseline > gpurun_out/ab_memo0b.log 2>&1" \
  "ESP_PLANES_DY_MEMO=1 timeout -k 10 300 python -u bench.py --config c5 --batch 64 --no-cpu-baseline > gpurun_out/ab_memo1b.log 2>&1"
