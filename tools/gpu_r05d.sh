#!/bin/bash
# round 5: probabilities kernel with two-step staging prefetch + KC x RC pipelined GEMMs: attention A/B
# vs the per-wave kernel (VARIANT=_w), attention PMC, bench twice, model parity
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_ANY"
rm -rf gpurun_out/pmc_d*
bash gpurun_steps.sh \
  "for v in '' _w; do for l in '' --legacy; do echo \"variant=\$v \$l\"; ESP_LIB_VARIANT=\$v timeout -k 10 120 python -u tools/attn_kernels_bench.py 256 --only probs \$l || exit 1; done; done > gpurun_out/r05d_attn_ab.txt 2>&1" \
  "timeout -s KILL 90 rocprofv3 --pmc $P1 -d gpurun_out/pmc_d1 -o run -- python3 tools/attn_kernels_bench.py 256 --only probs > gpurun_out/pmc_d1.log 2>&1" \
  "timeout -s KILL 90 rocprofv3 --pmc $P2 -d gpurun_out/pmc_d2 -o run -- python3 tools/attn_kernels_bench.py 256 --only probs > gpurun_out/pmc_d2.log 2>&1" \
  "timeout -k 10 600 python -u -m pytest tests/test_gpu_blocks.py tests/test_gpu_model.py tests/test_gpu_bench_shape.py -v -s --maxfail 10 --timeout 350 --timeout-method thread > gpurun_out/r05d_pytest.log 2>&1; rc=\$?; [ \$rc -le 1 ]" \
  "timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/r05d_bench.log 2>&1" \
  "timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/r05d_bench2.log 2>&1"
