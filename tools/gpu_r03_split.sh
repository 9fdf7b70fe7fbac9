#!/bin/bash
# Records for the bf16x6-split fp32 GEMM default: accuracy (split and f32-MFMA builds), GPU suite,
# default bench, rocprofv3 kernel summary, per-shape GEMM rates.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/prof
bash gpurun_steps.sh \
 "timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > gpurun_out/pytest_full.log 2>&1" \
 "timeout -k 10 200 python tools/f32_gemm_accuracy.py > gpurun_out/acc_split.log 2>&1" \
 "ESP_LIB_VARIANT=_f32 timeout -k 10 200 python tools/f32_gemm_accuracy.py > gpurun_out/acc_f32.log 2>&1" \
 "timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1" \
 "timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof.log 2>&1" \
 "timeout -k 10 200 python tools/gemm_profile.py --batch 128 > gpurun_out/gemm_shapes.log 2>&1" || exit $?
python3 tools/prof_summary.py gpurun_out/prof 8 > gpurun_out/kernel_summary_c2.txt 2>&1
rm -rf gpurun_out/prof
