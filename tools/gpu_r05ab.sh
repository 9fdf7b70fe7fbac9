#!/bin/bash
# round 5: conv1 forward without per-pixel divisions: parity (conv1 / subsampling / full-size / bench-shape), bench, kernel trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/prof_ab
bash gpurun_steps.sh \
  "timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_blocks.py tests/test_gpu_fullsize.py tests/test_gpu_bench_shape.py -k 'conv or subsampl or fullsize or bench_shape' -q --timeout 300 --timeout-method thread > gpurun_out/r05ab_pytest.log 2>&1" \
  "timeout -k 10 400 python -u bench.py --no-cpu-baseline --feed-steps 0 > gpurun_out/r05ab_bench.log 2>&1" \
  "timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ab -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --feed-steps 0 > gpurun_out/prof_ab.log 2>&1"
