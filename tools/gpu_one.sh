#!/bin/bash
# one-off GPU step list (edited per experiment): the whole GPU test suite at HEAD
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest.log 2>&1
