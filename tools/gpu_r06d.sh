#!/bin/bash
# round 6 (d): the whole GPU suite at HEAD (new parity gates: align_c2, fingerprints, trainrun vs fp64,
# dq_v band under split-K, batched forced-align, conv2d6, long utterances), smoke
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash gpurun_steps.sh \
  "timeout -k 10 1100 python -u -m pytest tests -m gpu -v -rf --timeout 350 --timeout-method thread > gpurun_out/r06d_pytest_gpu.log 2>&1" \
  "timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/r06d_smoke.log 2>&1"
