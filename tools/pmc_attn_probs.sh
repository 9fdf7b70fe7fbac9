#!/bin/bash
# PMC passes over the rel-pos probabilities kernel alone (tools/attn_kernels_bench.py --only probs, B=256):
# the block-staged kernel (default build) and the per-wave kernel (libespnet_mi355_w.so, VARIANT=_w)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_ANY"
P3="SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_IFETCH SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA"
rm -rf gpurun_out/pmc_ap*
steps=()
for v in lds _w; do
  lib=$v; [ "$v" = lds ] && lib=""
  for i in 1 2 3; do
    c=P$i
    steps+=("ESP_LIB_VARIANT=$lib timeout -s KILL 90 rocprofv3 --pmc ${!c} -d gpurun_out/pmc_ap${v}_$i -o run -- python3 tools/attn_kernels_bench.py 256 --only probs > gpurun_out/pmc_ap${v}_$i.log 2>&1")
  done
done
bash gpurun_steps.sh "${steps[@]}"
