#!/bin/bash
# round 4 GPU step list (edited per experiment)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash gpurun_steps.sh \
  "timeout -k 10 700 python -u tests/golden/make_bench_fixture.py gpurun_out/bench_c2_b128.npz > gpurun_out/bench_fixture_gen.log 2>&1" \
  "cp gpurun_out/bench_c2_b128.npz tests/golden/bench_c2_b128.npz" \
  "timeout -k 10 900 python -u -m pytest -v tests/test_gpu_fullsize.py tests/test_gpu_bench_shape.py tests/test_slurp_config.py tests/test_gpu_distributed.py tests/test_gpu_trainrun.py --timeout 400 --timeout-method thread > gpurun_out/pytest_r04a.log 2>&1"
