#!/bin/bash
# round 5: the B=384 bench shape against the oracle fixture (three copies) before the default batch moves
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash gpurun_steps.sh \
  "timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_shape.py -k b256 -v -s --timeout 500 --timeout-method thread > gpurun_out/r05w_pytest_b384.log 2>&1"
