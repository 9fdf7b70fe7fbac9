#!/bin/bash
# round 4: the dy bf16 copy handed over in the planes GEMM path -- bf16 / C5 tests, cast census, C5 bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash gpurun_steps.sh \
  "timeout -k 10 600 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_fullsize.py -m gpu -v --timeout 250 --timeout-method thread > gpurun_out/pytest_memo.log 2>&1" \
  "timeout -k 10 300 python -u tools/cast_census.py --batch 64 > gpurun_out/cast_census_c5_memo.txt 2>&1" \
  "timeout -k 10 400 python -u bench.py --config c5 --batch 64 --no-cpu-baseline > gpurun_out/bench_c5_memo.log 2>&1"
