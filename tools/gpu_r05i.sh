#!/bin/bash
# round 5: PMC of the weight-gradient GEMM (RC x RC, PREC 0, fused row sums) and a KC x RC PREC 0 GEMM of the
# same size, one shape each (tools/gemm_one.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_MISC SQ_BUSY_CYCLES"
rm -rf gpurun_out/pmc_w*
bash gpurun_steps.sh \
  "timeout -k 10 120 python -u tools/gemm_one.py 1 1 1024 256 95744 20 --rowsum > gpurun_out/r05i_gemm_one.txt 2>&1 && timeout -k 10 120 python -u tools/gemm_one.py 0 1 95744 256 1024 20 >> gpurun_out/r05i_gemm_one.txt 2>&1 && timeout -k 10 120 python -u tools/gemm_one.py 1 1 256 256 95744 20 --rowsum >> gpurun_out/r05i_gemm_one.txt 2>&1" \
  "timeout -s KILL 90 rocprofv3 --pmc $P1 -d gpurun_out/pmc_w1 -o run -- python3 tools/gemm_one.py 1 1 1024 256 95744 5 --rowsum > gpurun_out/pmc_w1.log 2>&1" \
  "timeout -s KILL 90 rocprofv3 --pmc $P2 -d gpurun_out/pmc_w2 -o run -- python3 tools/gemm_one.py 1 1 1024 256 95744 5 --rowsum > gpurun_out/pmc_w2.log 2>&1" \
  "timeout -s KILL 90 rocprofv3 --pmc $P1 -d gpurun_out/pmc_wk1 -o run -- python3 tools/gemm_one.py 0 1 95744 256 1024 5 > gpurun_out/pmc_wk1.log 2>&1" \
  "timeout -s KILL 90 rocprofv3 --pmc $P2 -d gpurun_out/pmc_wk2 -o run -- python3 tools/gemm_one.py 0 1 95744 256 1024 5 > gpurun_out/pmc_wk2.log 2>&1"
