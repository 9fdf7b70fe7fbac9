#!/bin/bash
# round 5 first records: the whole GPU suite (loss-gate errors printed), the C2 bench, its kernel summary
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/prof
bash gpurun_steps.sh \
  "timeout -k 10 1200 python -u -m pytest tests -m gpu -v -s --maxfail 15 --timeout 350 --timeout-method thread > gpurun_out/r05a_pytest_gpu.log 2>&1; rc=\$?; [ \$rc -le 1 ]" \
  "timeout -k 10 400 python -u bench.py > gpurun_out/r05a_bench.log 2>&1" \
  "timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof.log 2>&1"
