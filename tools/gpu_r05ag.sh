#!/bin/bash
# round 5: score-row pitch granularity (kernels.SCORE_ALIGN 4 -> 32 floats: 128-B aligned P / dS / dbd rows)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/prof_ag
bash gpurun_steps.sh \
  "timeout -k 10 400 python -u bench.py --no-cpu-baseline --feed-steps 0 > gpurun_out/r05ag_bench.log 2>&1" \
  "timeout -k 10 400 python -u tools/bench_with.py kernels.SCORE_ALIGN=32 -- --no-cpu-baseline --feed-steps 0 > gpurun_out/r05ag_bench_a32.log 2>&1" \
  "timeout -k 10 400 python -u bench.py --no-cpu-baseline --feed-steps 0 > gpurun_out/r05ag_bench2.log 2>&1" \
  "timeout -k 10 400 python -u tools/bench_with.py kernels.SCORE_ALIGN=32 -- --no-cpu-baseline --feed-steps 0 > gpurun_out/r05ag_bench_a32b.log 2>&1" \
  "timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ag -o run -- python3 tools/bench_with.py kernels.SCORE_ALIGN=32 -- --steps 5 --warmup 2 --no-cpu-baseline --feed-steps 0 > gpurun_out/prof_ag.log 2>&1"
