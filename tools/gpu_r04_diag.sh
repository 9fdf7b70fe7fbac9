#!/bin/bash
# round 4 diagnostics: C5 cast census, C2 per-shape GEMM device times from a kernel trace, the pending B=256 check
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/prof_shapes
bash gpurun_steps.sh \
  "timeout -k 10 300 python -u tools/cast_census.py --batch 64 > gpurun_out/cast_census_c5.txt 2>&1" \
  "timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_shapes -o run -- python3 tools/gemm_profile.py --batch 128 --order gpurun_out/gemm_order_b128.tsv > gpurun_out/gemm_profile_b128.log 2>&1" \
  "python3 tools/gemm_shapes_trace.py gpurun_out/prof_shapes gpurun_out/gemm_order_b128.tsv > gpurun_out/gemm_shapes_trace_b128.txt 2>&1" \
  "rm -rf gpurun_out/prof_shapes" \
  "timeout -k 10 400 python -u -m pytest tools/pending_b256_check.py -v --timeout 350 --timeout-method thread > gpurun_out/pytest_b256.log 2>&1"
