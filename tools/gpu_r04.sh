#!/bin/bash
# round 4 GPU step list (edited per experiment)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/pmc_ap*
bash gpurun_steps.sh \
  "timeout -k 10 300 python -u -m pytest tests/test_gpu_blocks.py tests/test_gpu_kernels.py -x -q -k 'relpos or mha or attn' --timeout 120 --timeout-method thread > gpurun_out/pytest_attn.log 2>&1" \
  "ESP_ATTN_XS=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_blocks.py -x -q -k 'relpos' --timeout 120 --timeout-method thread > gpurun_out/pytest_attn_xs.log 2>&1" \
  "timeout -k 10 120 python -u tools/attn_kernels_bench.py 128 --only probs > gpurun_out/attn_f32.log 2>&1" \
  "ESP_ATTN_XS=1 timeout -k 10 120 python -u tools/attn_kernels_bench.py 128 --only probs > gpurun_out/attn_xs.log 2>&1" \
  "timeout -k 10 120 python -u tools/attn_kernels_bench.py 128 --only probs --legacy > gpurun_out/attn_f32_leg.log 2>&1" \
  "ESP_ATTN_XS=1 timeout -k 10 120 python -u tools/attn_kernels_bench.py 128 --only probs --legacy > gpurun_out/attn_xs_leg.log 2>&1" \
  "timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_ANY -d gpurun_out/pmc_ap0_2 -o run -- python3 tools/attn_kernels_bench.py 128 --only probs > gpurun_out/pmc_ap0_2.log 2>&1"
