#!/bin/bash
# round 5: per-shape GEMM device time of one eager C2 B=256 step at HEAD (kernel trace mapped onto the launch order)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/prof_ai
bash gpurun_steps.sh \
  "timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_ai -o run -- python3 tools/gemm_profile.py --batch 256 --order gpurun_out/r05ai_order.tsv > gpurun_out/r05ai_gemm_profile.log 2>&1"
