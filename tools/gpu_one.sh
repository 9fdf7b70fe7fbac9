cd "${GRAFT_REPO_ROOT}"
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "dropout" -x -v --timeout 120 --timeout-method thread > gpurun_out/pt_drop.log 2>&1
