#!/bin/bash
# round 5: LayerNorm outputs with their split planes for the weight gradients (PREC 3 RC x RC): parity, bench A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/prof_j
bash gpurun_steps.sh \
  "timeout -k 10 700 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_bench_shape.py tests/test_gpu_fullsize.py tests/test_gpu_trainer.py tests/test_gpu_trainrun.py tests/test_gpu_distributed.py -v -s --maxfail 10 --timeout 350 --timeout-method thread > gpurun_out/r05j_pytest.log 2>&1; rc=\$?; [ \$rc -le 1 ]" \
  "timeout -k 10 400 python -u bench.py --no-cpu-baseline --feed-steps 0 > gpurun_out/r05j_bench.log 2>&1" \
  "timeout -k 10 400 python -u tools/bench_with.py kernels.WGRAD_XPLANES=0 -- --no-cpu-baseline --feed-steps 0 > gpurun_out/r05j_bench_off.log 2>&1" \
  "timeout -k 10 400 python -u bench.py --no-cpu-baseline --feed-steps 0 > gpurun_out/r05j_bench2.log 2>&1" \
  "timeout -k 10 400 python -u tools/bench_with.py kernels.WGRAD_XPLANES=0 -- --no-cpu-baseline --feed-steps 0 > gpurun_out/r05j_bench_off2.log 2>&1" \
  "timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_j -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --feed-steps 0 > gpurun_out/prof_j.log 2>&1"
