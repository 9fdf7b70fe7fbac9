#!/bin/bash
# round 5: the split residuals as v_dot2c_f32_bf16 (ESP_SPLIT_DOT=1, default build) vs the unpack + v_sub
# form (libespnet_mi355_nodot.so): parity, GEMM timings, bench A/B, kernel summary
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/prof_n
T=gpurun_out/r05n_gemm.txt
bash gpurun_steps.sh \
  "timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py::test_f32_to_planes_exact_split tests/test_gpu_kernels.py -k 'planes_exact or f32_accuracy or b_planes_bit_exact' -x -v -s --timeout 120 --timeout-method thread > gpurun_out/r05n_pytest0.log 2>&1" \
  "timeout -k 10 700 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_bench_shape.py tests/test_gpu_fullsize.py tests/test_gpu_blocks.py -v -s --maxfail 10 --timeout 350 --timeout-method thread > gpurun_out/r05n_pytest.log 2>&1" \
  "for v in '' _nodot; do for s in '1 1 1024 256 95744 20 --rowsum' '1 1 256 256 95744 20 --rowsum' '0 1 95744 256 1024 20 --bw' '0 0 95744 1024 256 20 --bw'; do ESP_LIB_VARIANT=\$v timeout -k 10 60 python -u tools/gemm_one.py \$s >> $T 2>&1 || exit 1; echo \"  [\$v]\" >> $T; done; done" \
  "timeout -k 10 400 python -u bench.py --no-cpu-baseline --feed-steps 0 > gpurun_out/r05n_bench.log 2>&1" \
  "ESP_LIB_VARIANT=_nodot timeout -k 10 400 python -u bench.py --no-cpu-baseline --feed-steps 0 > gpurun_out/r05n_bench_nd.log 2>&1" \
  "timeout -k 10 400 python -u bench.py --no-cpu-baseline --feed-steps 0 > gpurun_out/r05n_bench2.log 2>&1" \
  "ESP_LIB_VARIANT=_nodot timeout -k 10 400 python -u bench.py --no-cpu-baseline --feed-steps 0 > gpurun_out/r05n_bench_nd2.log 2>&1" \
  "timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_n -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --feed-steps 0 > gpurun_out/prof_n.log 2>&1"
