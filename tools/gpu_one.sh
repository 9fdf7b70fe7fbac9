#!/bin/bash
# one-off GPU step runner: the command in $ONE_CMD-free form below is edited per experiment
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 300 python -u tools/gemm_profile.py --batch 128 > gpurun_out/gemm_shapes.log 2>&1
