#!/bin/bash
# round 5: FusedAdam param groups + amsgrad on the GPU (ABI 30), and the trainer / checkpoint / kernel tests around it
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash gpurun_steps.sh \
  "timeout -k 10 600 python -u -m pytest tests/test_gpu_optim.py tests/test_gpu_trainer.py tests/test_gpu_checkpoint.py tests/test_gpu_trainrun.py tests/test_gpu_graph.py -k 'not nothing' -v --timeout 300 --timeout-method thread > gpurun_out/r05aa_pytest_optim.log 2>&1" \
  "timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py -k adam -q --timeout 120 --timeout-method thread >> gpurun_out/r05aa_pytest_optim.log 2>&1"
