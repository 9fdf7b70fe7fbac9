#!/bin/bash
# round 5: 64 x 64 tiles weighed against 128-wide ones for unsplit grids (ESP_GEMM_BM64_ANY=1, 64x64 cost 0.6,
# libespnet_mi355_b64.so) vs the default model: decoder-side shapes, per-shape trace, bench A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=gpurun_out/r05al_gemm.txt
rm -f $T
rm -rf gpurun_out/prof_al
bash gpurun_steps.sh \
  "ESP_LIB_VARIANT=_b64 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k 'gemm' -x -q --timeout 120 --timeout-method thread > gpurun_out/r05al_pytest_b64.log 2>&1" \
  "for v in '' _b64; do for s in '0 0 10496 256 256 20' '0 1 10496 256 256 20' '0 0 10496 2048 256 20' '0 0 10496 256 2048 20' '0 0 95744 256 256 20'; do ESP_LIB_VARIANT=\$v timeout -k 10 60 python -u tools/gemm_one.py \$s --bw >> $T 2>&1 || exit 1; echo \"  [\$v] \$s\" >> $T; done; done" \
  "timeout -k 10 400 python -u bench.py --no-cpu-baseline --feed-steps 0 > gpurun_out/r05al_bench.log 2>&1" \
  "ESP_LIB_VARIANT=_b64 timeout -k 10 400 python -u bench.py --no-cpu-baseline --feed-steps 0 > gpurun_out/r05al_bench_b64.log 2>&1" \
  "timeout -k 10 400 python -u bench.py --no-cpu-baseline --feed-steps 0 > gpurun_out/r05al_bench2.log 2>&1" \
  "ESP_LIB_VARIANT=_b64 timeout -k 10 400 python -u bench.py --no-cpu-baseline --feed-steps 0 > gpurun_out/r05al_bench_b64b.log 2>&1"
