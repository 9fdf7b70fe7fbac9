#!/bin/bash
# one-off GPU step list (edited per experiment): smoke, legacy rel-pos and C5 bench lines at HEAD
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash gpurun_steps.sh \
  "timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")' > gpurun_out/smoke.log 2>&1" \
  "timeout -k 10 300 python -u bench.py --rel-pos legacy --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_legacy.log 2>&1" \
  "timeout -k 10 300 python -u bench.py --config c5 --batch 64 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_c5_b64.log 2>&1"
