#!/bin/bash
# round 4: same-box A/B of the split-K minimum chunk (ESP_SPLITK_MINK 128 = before, 256 = new default),
# C2 B=256 and C5 B=64 alternating, the per-shape trace at the new default, then the whole GPU suite
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/prof_shapes
bash gpurun_steps.sh \
  "ESP_SPLITK_MINK=128 timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/ab_mink128a.log 2>&1" \
  "ESP_SPLITK_MINK=256 timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/ab_mink256a.log 2>&1" \
  "ESP_SPLITK_MINK=128 timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/ab_mink128b.log 2>&1" \
  "ESP_SPLITK_MINK=256 timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/ab_mink256b.log 2>&1" \
  "ESP_SPLITK_MINK=128 timeout -k 10 300 python -u bench.py --config c5 --batch 64 --no-cpu-baseline > gpurun_out/ab_mink128_c5.log 2>&1" \
  "ESP_SPLITK_MINK=256 timeout -k 10 300 python -u bench.py --config c5 --batch 64 --no-cpu-baseline > gpurun_out/ab_mink256_c5.log 2>&1" \
  "timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_shapes -o run -- python3 tools/gemm_profile.py --batch 128 --order gpurun_out/gemm_order_b128.tsv > gpurun_out/gemm_profile_b128.log 2>&1" \
  "python3 tools/gemm_shapes_trace.py gpurun_out/prof_shapes gpurun_out/gemm_order_b128.tsv > gpurun_out/gemm_shapes_trace_b128_mink256.txt 2>&1" \
  "rm -rf gpurun_out/prof_shapes" \
  "timeout -k 10 1500 python -u -m pytest tests -m gpu -v --timeout 350 --timeout-method thread > gpurun_out/pytest_gpu_all.log 2>&1"
