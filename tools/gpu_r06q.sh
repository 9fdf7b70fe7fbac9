#!/bin/bash
# round 6 (q): batch A/B at HEAD -- C2 B=256 vs B=384 alternating (1-GPU graph step), then the DP path at B=384
# (HBM per rank for the 8-GPU run)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash gpurun_steps.sh \
  "for b in 256 384 256 384; do echo \"batch=\$b\"; timeout -k 10 400 python -u bench.py --batch \$b --no-cpu-baseline --feed-steps 0 --steps 20 | tail -1 || exit 1; done > gpurun_out/r06q_batch_ab.log 2>&1" \
  "timeout -k 10 400 python -u bench.py --dp-world1 --batch 384 --no-cpu-baseline --feed-steps 0 --steps 10 > gpurun_out/r06q_bench_dp_b384.log 2>&1"
