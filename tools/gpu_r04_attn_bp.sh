#!/bin/bash
# round 4: batched attention contractions on B planes (ESP_ATTN_BPLANES=1) -- parity tests with it on,
# same-box A/B at C2 B=256 (alternating), per-shape trace with it on
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/prof_shapes
bash gpurun_steps.sh \
  "ESP_ATTN_BPLANES=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_bench_shape.py tests/test_gpu_blocks.py tests/test_gpu_model.py -m gpu -v --timeout 350 --timeout-method thread > gpurun_out/pytest_attn_bp.log 2>&1" \
  "ESP_ATTN_BPLANES=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/ab_bp0a.log 2>&1" \
  "ESP_ATTN_BPLANES=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/ab_bp1a.log 2>&1" \
  "ESP_ATTN_BPLANES=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/ab_bp0b.log 2>&1" \
  "ESP_ATTN_BPLANES=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/ab_bp1b.log 2>&1" \
  "ESP_ATTN_BPLANES=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_shapes -o run -- python3 tools/gemm_profile.py --batch 128 --order gpurun_out/gemm_order_b128.tsv > gpurun_out/gemm_profile_b128.log 2>&1" \
  "python3 tools/gemm_shapes_trace.py gpurun_out/prof_shapes gpurun_out/gemm_order_b128.tsv > gpurun_out/gemm_shapes_trace_b128_bp.txt 2>&1" \
  "rm -rf gpurun_out/prof_shapes"
