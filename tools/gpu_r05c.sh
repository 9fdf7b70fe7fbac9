#!/bin/bash
# round 5: pipelined GEMM k-loop -- GEMM / model parity, bench A/B vs the round-4 k-loop (VARIANT=_np),
# per-kernel times of both, PMC of the probabilities kernels
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/prof_c gpurun_out/prof_np
bash gpurun_steps.sh \
  "timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_bench_shape.py tests/test_gpu_fullsize.py tests/test_slurp_config.py -v -s --maxfail 10 --timeout 350 --timeout-method thread > gpurun_out/r05c_pytest.log 2>&1; rc=\$?; [ \$rc -le 1 ]" \
  "timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/r05c_bench.log 2>&1" \
  "ESP_LIB_VARIANT=_np timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/r05c_bench_np.log 2>&1" \
  "timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/r05c_bench2.log 2>&1" \
  "ESP_LIB_VARIANT=_np timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/r05c_bench_np2.log 2>&1" \
  "timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_c.log 2>&1" \
  "ESP_LIB_VARIANT=_np timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_np -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_np.log 2>&1" \
  "bash tools/pmc_attn_probs.sh > gpurun_out/pmc_attn.log 2>&1"
