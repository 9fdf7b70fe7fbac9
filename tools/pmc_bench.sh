#!/bin/bash
# SQ counter passes over a short bench run (per-kernel MFMA busy, VALU / LDS / wait cycles)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
rm -rf gpurun_out/pmcb1 gpurun_out/pmcb2
bash gpurun_steps.sh \
 "timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA -d gpurun_out/pmcb1 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --eager > gpurun_out/pmcb1.log 2>&1" \
 "timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_INSTS_SALU -d gpurun_out/pmcb2 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --eager > gpurun_out/pmcb2.log 2>&1" || exit $?
# the rocpd databases exceed what gpurun copies back: summarise on the box, keep only the text
python3 tools/pmc_kernel.py gpurun_out/pmcb1 gpurun_out/pmcb2 > gpurun_out/pmcb_summary.txt 2>&1
rm -rf gpurun_out/pmcb1 gpurun_out/pmcb2
