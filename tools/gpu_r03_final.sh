#!/bin/bash
# Round-3 HEAD records: full GPU suite (verbatim log), smoke(), default bench (with cpu_baseline),
# C5 line, rocprofv3 kernel summary of the C2 step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/prof
bash gpurun_steps.sh \
 "timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > gpurun_out/pytest_full.log 2>&1" \
 "timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/smoke.log 2>&1" \
 "timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1" \
 "timeout -k 10 300 python bench.py --config c5 --batch 64 --no-cpu-baseline > gpurun_out/bench_c5.log 2>&1" \
 "timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof.log 2>&1" || exit $?
python3 tools/prof_summary.py gpurun_out/prof 8 > gpurun_out/kernel_summary_c2.txt 2>&1
rm -rf gpurun_out/prof
