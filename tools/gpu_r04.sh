#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash gpurun_steps.sh "timeout -k 10 200 python -u tools/quant_bench.py > gpurun_out/quant.log 2>&1"
