set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > gpurun_out/r02a_pytest_gpu.log 2>&1
