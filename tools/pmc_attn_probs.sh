#!/bin/bash
# PMC passes over the rel-pos probabilities kernel alone (tools/attn_kernels_bench.py --only probs),
# f32-MFMA form and split-product form (ESP_ATTN_XS=1)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_ANY"
P3="SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_IFETCH SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA"
rm -rf gpurun_out/pmc_ap*
steps=()
for xs in 0 1; do
  for i in 1 2 3; do
    v=P$i
    steps+=("ESP_ATTN_XS=$xs timeout -s KILL 90 rocprofv3 --pmc ${!v} -d gpurun_out/pmc_ap${xs}_$i -o run -- python3 tools/attn_kernels_bench.py 128 --only probs > gpurun_out/pmc_ap${xs}_$i.log 2>&1")
  done
done
bash gpurun_steps.sh "${steps[@]}"
