#!/bin/bash
# round 6 (k): final HEAD record -- the full GPU suite (-s), smoke, the default bench line (cpu_baseline leg
# included), the legacy bench line, a C2 B=256 kernel trace and the GEMM-family HBM traffic (two --pmc passes)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/prof_k
bash gpurun_steps.sh \
  "timeout -k 10 1100 python -u -m pytest tests -m gpu -v -s -rf --timeout 350 --timeout-method thread > gpurun_out/r06k_pytest_gpu.log 2>&1" \
  "timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/r06k_smoke.log 2>&1" \
  "timeout -k 10 500 python -u bench.py > gpurun_out/r06k_bench.log 2>&1" \
  "timeout -k 10 300 python -u bench.py --rel-pos legacy --no-cpu-baseline --feed-steps 0 > gpurun_out/r06k_bench_legacy.log 2>&1" \
  "timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_k -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --feed-steps 0 > gpurun_out/prof_k.log 2>&1" \
  "bash tools/pmc_traffic.sh > gpurun_out/pmc_c2_k.log 2>&1"
