#!/bin/bash
# round 5 records at HEAD: the whole GPU suite + smoke, the C2 bench (with the data-feed rate), its kernel summary
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/prof_ar
bash gpurun_steps.sh \
  "timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 350 --timeout-method thread > gpurun_out/r05ar_pytest_gpu.log 2>&1" \
  "timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/r05ar_smoke.log 2>&1" \
  "timeout -k 10 400 python -u bench.py > gpurun_out/r05ar_bench.log 2>&1" \
  "timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ar -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --feed-steps 0 > gpurun_out/prof_ar.log 2>&1"
