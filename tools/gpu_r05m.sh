#!/bin/bash
# round 5: weight-gradient GEMM (RC x RC, row sums) at PREC 0 / 3 (B planes) / 5 (both planes): timings
# at the C2 B=256 shapes, then SQ PMC passes of PREC 0 and PREC 5 at the FFN w_1 shape
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_MISC SQ_BUSY_CYCLES"
rm -rf gpurun_out/pmc_m*
T=gpurun_out/r05m_wgrad.txt
S="1024 256 95744"
bash gpurun_steps.sh \
  "for s in '1024 256 95744' '256 1024 95744' '256 256 95744' '768 256 95744'; do for f in '' '--bw' '--pl'; do timeout -k 10 60 python -u tools/gemm_one.py 1 1 \$s 20 --rowsum \$f >> $T 2>&1 || exit 1; echo \"  [\$f]\" >> $T; done; done" \
  "timeout -s KILL 90 rocprofv3 --pmc $P1 -d gpurun_out/pmc_m1 -o run -- python3 tools/gemm_one.py 1 1 $S 5 --rowsum > gpurun_out/pmc_m1.log 2>&1" \
  "timeout -s KILL 90 rocprofv3 --pmc $P2 -d gpurun_out/pmc_m2 -o run -- python3 tools/gemm_one.py 1 1 $S 5 --rowsum > gpurun_out/pmc_m2.log 2>&1" \
  "timeout -s KILL 90 rocprofv3 --pmc $P1 -d gpurun_out/pmc_m3 -o run -- python3 tools/gemm_one.py 1 1 $S 5 --rowsum --pl > gpurun_out/pmc_m3.log 2>&1" \
  "timeout -s KILL 90 rocprofv3 --pmc $P2 -d gpurun_out/pmc_m4 -o run -- python3 tools/gemm_one.py 1 1 $S 5 --rowsum --pl > gpurun_out/pmc_m4.log 2>&1"
