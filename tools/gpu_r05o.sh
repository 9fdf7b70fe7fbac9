#!/bin/bash
# round 5: GEMM bound analysis: default vs diagnostic builds _a1 (no next-slab LDS-DMA: compute on stale
# slabs, barriers kept) and _a5 (no DMA, no waits / barriers: the k-loop's LDS reads + split + MFMAs alone)
# _a128: the split reduced to the hi cast (mid = lo = hi), _a133: that without DMA / barriers
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=gpurun_out/r05o_gemm_abl.txt
rm -f $T
bash gpurun_steps.sh \
  "for v in '' _ig0; do for s in '1 1 1024 256 95744 20 --rowsum' '1 1 256 256 95744 20 --rowsum' '0 1 95744 256 1024 20 --bw' '0 0 95744 1024 256 20 --bw' '0 0 95744 1024 256 20'; do ESP_LIB_VARIANT=\$v timeout -k 10 60 python -u tools/gemm_one.py \$s >> $T 2>&1 || exit 1; echo \"  [\$v] \$s\" >> $T; done; done"
