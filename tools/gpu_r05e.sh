#!/bin/bash
# round 5: probabilities kernel with 3 staging steps in flight: attention microbench, C2 bench, C5 bench +
# its kernel summary (the bf16 mode's single-product form of the new kernel)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/prof_c5e
bash gpurun_steps.sh \
  "for l in '' --legacy; do echo \"PF=3 \$l\"; timeout -k 10 120 python -u tools/attn_kernels_bench.py 256 --only probs \$l || exit 1; done > gpurun_out/r05e_attn.txt 2>&1" \
  "timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/r05e_bench.log 2>&1" \
  "timeout -k 10 400 python -u bench.py --config c5 --batch 64 --no-cpu-baseline > gpurun_out/r05e_bench_c5.log 2>&1" \
  "timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5e -o run -- python3 bench.py --config c5 --batch 64 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_c5e.log 2>&1" \
  "timeout -k 10 600 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_blocks.py tests/test_gpu_fullsize.py -v -s --maxfail 10 --timeout 350 --timeout-method thread > gpurun_out/r05e_pytest.log 2>&1; rc=\$?; [ \$rc -le 1 ]"
