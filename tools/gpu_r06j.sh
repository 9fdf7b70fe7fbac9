#!/bin/bash
# round 6 (j): non-temporal P / P_drop stores in the probabilities kernel (_nt) vs the default build --
# probabilities microbench (latest / legacy), then alternating C2 B=256 bench lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash gpurun_steps.sh \
  "for v in '' _nt '' _nt; do for l in '' --legacy; do echo \"lib=\$v \$l\"; ESP_LIB_VARIANT=\$v timeout -k 10 120 python -u tools/attn_kernels_bench.py 256 --only probs \$l || exit 1; done; done > gpurun_out/r06j_probs.log 2>&1" \
  "for v in '' _nt '' _nt; do echo \"lib=\$v\"; ESP_LIB_VARIANT=\$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --feed-steps 0 --steps 20 | tail -1 || exit 1; done > gpurun_out/r06j_bench_ab.log 2>&1"
