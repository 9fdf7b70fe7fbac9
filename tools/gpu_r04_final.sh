#!/bin/bash
# round 4 final records at HEAD (bench default B=256): the whole GPU suite + smoke, the C2 bench, its rocprof
# kernel summary and GEMM-family HBM traffic
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/prof
bash gpurun_steps.sh \
  "timeout -k 10 1500 python -u -m pytest tests -m gpu -v --timeout 350 --timeout-method thread > gpurun_out/pytest_gpu_all.log 2>&1" \
  "timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/smoke.log 2>&1" \
  "timeout -k 10 400 python -u bench.py > gpurun_out/bench_head.log 2>&1" \
  "timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof.log 2>&1" \
  "TAG=c2 bash tools/pmc_traffic.sh > gpurun_out/pmc_c2.log 2>&1"
