#!/bin/bash
# full GPU iteration: every GPU test, the attention microbench, the default bench line and a
# rocprofv3 kernel trace of a short bench run (each step under its own limit; stops at the first failure)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
rm -rf gpurun_out/prof
bash gpurun_steps.sh \
  "timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest.log 2>&1" \
  "timeout -k 10 120 python -u tools/attn_bench.py 128 --fwd-only > gpurun_out/attn_bench.log 2>&1" \
  "timeout -k 10 400 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1" \
  "timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/prof.log 2>&1"
