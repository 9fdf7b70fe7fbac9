#!/bin/bash
# round 5: conv1 forward with non-temporal stores (ESP_CONV1_NT=1, libespnet_mi355_nt.so) vs plain stores: kernel traces
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/prof_ac gpurun_out/prof_acn
bash gpurun_steps.sh \
  "timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ac -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --feed-steps 0 > gpurun_out/prof_ac.log 2>&1" \
  "ESP_LIB_VARIANT=_nt timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_acn -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --feed-steps 0 > gpurun_out/prof_acn.log 2>&1"
