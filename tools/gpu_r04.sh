#!/bin/bash
# round 4 GPU step list (edited per experiment)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/prof gpurun_out/prof_c5
bash gpurun_steps.sh \
  "timeout -k 10 600 python -u -m pytest tests/test_gpu_distributed.py tests/test_gpu_graph.py tests/test_gpu_fullsize.py -v -x --timeout 170 --timeout-method thread > gpurun_out/pytest_full.log 2>&1" \
  "timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof.log 2>&1" \
  "timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5 -o run -- python3 bench.py --config c5 --batch 64 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_c5.log 2>&1" \
  "timeout -k 10 200 python3 tools/gemm_profile.py --batch 128 > gpurun_out/gemm_shapes_c2.txt 2>&1" \
  "timeout -k 10 200 python3 tools/gemm_profile.py --batch 64 --config c5 > gpurun_out/gemm_shapes_c5.txt 2>&1"
