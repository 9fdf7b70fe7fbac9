#!/bin/bash
# PMC passes over the GEMM kernel: ffn w1 dX shape (KC x RC, 47872 x 256 x 1024), in-register split vs B planes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_ANY"
P3="SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_IFETCH"
steps=()
for bp in 0 1; do
  for i in 1 2 3; do
    v=P$i
    steps+=("timeout -s KILL 90 rocprofv3 --pmc ${!v} -d gpurun_out/pmc_bp${bp}_$i -o run -- python3 tools/bp_bench.py 3 $bp 5 > gpurun_out/pmc_bp${bp}_$i.log 2>&1")
  done
done
bash gpurun_steps.sh "${steps[@]}"
