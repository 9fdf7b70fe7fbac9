set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_flash.py tests/test_gpu_blocks.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/r02e_flash_tests.log 2>&1
