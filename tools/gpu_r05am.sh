#!/bin/bash
# round 5: per-kernel comparison of the 2-slab 256 x 128 / 8-wave tiles (libespnet_mi355_w2.so) vs default, kernel traces
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/prof_am gpurun_out/prof_amw
bash gpurun_steps.sh \
  "timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_am -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --feed-steps 0 > gpurun_out/prof_am.log 2>&1" \
  "ESP_LIB_VARIANT=_w2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_amw -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --feed-steps 0 > gpurun_out/prof_amw.log 2>&1"
