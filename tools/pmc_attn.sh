#!/bin/bash
# PMC passes over the fused attention-probability kernels (tools/attn_bench.py --fwd-only)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash gpurun_steps.sh \
 "timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA -d gpurun_out/pmc_att1 -o run -- python3 tools/attn_bench.py 128 --fwd-only > gpurun_out/pmc_att1.log 2>&1" \
 "timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_ANY -d gpurun_out/pmc_att2 -o run -- python3 tools/attn_bench.py 128 --fwd-only > gpurun_out/pmc_att2.log 2>&1" \
 "timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_IFETCH -d gpurun_out/pmc_att3 -o run -- python3 tools/attn_bench.py 128 --fwd-only > gpurun_out/pmc_att3.log 2>&1"
