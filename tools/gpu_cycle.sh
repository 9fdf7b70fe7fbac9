#!/bin/bash
# One GPU iteration: GPU parity tests, the default bench line, and a rocprofv3 kernel trace of a
# short bench run (all under their own time limits; stops at the first fault/timeout).
# usage: bash tools/gpu_cycle.sh [pytest-args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
rm -rf gpurun_out/prof
PYT=${PYT:-"tests -m gpu"}
bash gpurun_steps.sh \
  "timeout -k 10 600 python -u -m pytest $PYT -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest.log 2>&1" \
  "timeout -k 10 400 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1" \
  "export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/prof.log 2>&1"
