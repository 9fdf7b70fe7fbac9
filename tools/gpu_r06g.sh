#!/bin/bash
# round 6 (g): the legacy probabilities kernel with a branch-free shifted-row select (main: register fragment
# select, _va: LDS re-read select), conv1's bit map packed with DPP; tests, probabilities microbench, C2 B=256
# kernel traces (legacy, latest) and bench lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/prof_g_leg gpurun_out/prof_g_lat
bash gpurun_steps.sh \
  "timeout -k 10 500 python -u -m pytest tests/test_gpu_blocks.py tests/test_gpu_kernels.py -m gpu -v -rf -k 'relpos or probs or conv' --timeout 120 --timeout-method thread > gpurun_out/r06g_pytest.log 2>&1" \
  "for v in '' _va; do for l in '' --legacy; do echo \"lib=\$v \$l\"; ESP_LIB_VARIANT=\$v timeout -k 10 120 python -u tools/attn_kernels_bench.py 256 --only probs \$l || exit 1; done; done > gpurun_out/r06g_probs.log 2>&1" \
  "timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_g_leg -o run -- python3 bench.py --rel-pos legacy --steps 5 --warmup 2 --no-cpu-baseline --feed-steps 0 > gpurun_out/prof_g_leg.log 2>&1" \
  "timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_g_lat -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --feed-steps 0 > gpurun_out/prof_g_lat.log 2>&1" \
  "timeout -k 10 300 python -u bench.py --no-cpu-baseline --feed-steps 0 --steps 20 > gpurun_out/r06g_bench.log 2>&1" \
  "timeout -k 10 300 python -u bench.py --rel-pos legacy --no-cpu-baseline --feed-steps 0 --steps 20 > gpurun_out/r06g_bench_legacy.log 2>&1"
