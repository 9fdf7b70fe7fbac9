#!/bin/bash
# round 6 (u): where the implicit conv2 input gradient's per-class fixed cost goes -- the fold alone at C2 B=256
# under a kernel trace: default, _ab1 (epilogue does nothing), _ab2 (no conv1-input patch loads)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/prof_u0 gpurun_out/prof_u1 gpurun_out/prof_u2
bash gpurun_steps.sh \
  "timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_u0 -o run -- python3 tools/c1fold_bench.py > gpurun_out/r06u_c1fold.log 2>&1" \
  "ESP_LIB_VARIANT=_ab1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_u1 -o run -- python3 tools/c1fold_bench.py > gpurun_out/r06u_c1fold_ab1.log 2>&1" \
  "ESP_LIB_VARIANT=_ab2 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_u2 -o run -- python3 tools/c1fold_bench.py > gpurun_out/r06u_c1fold_ab2.log 2>&1"
