#!/bin/bash
# round 6 (f): (1) legacy probabilities kernel without VGPR spills (shifted q_v rows parked in LDS; _a2: legacy
# prefetch depth 2 too); (2) the conv2 input gradient's ReLU mask from conv1's packed bit map
# (esp_conv1_fwd_bits / esp_conv2_dgrad_bits; ESP_CONV2_BITS=0: the fp32 map).  Attention + conv kernel tests,
# then C2 B=256 kernel traces: legacy on the new build (bits on) and on _a2 (bits off), latest (bits on)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/prof_f_leg gpurun_out/prof_f_leg_a2 gpurun_out/prof_f_lat
bash gpurun_steps.sh \
  "timeout -k 10 500 python -u -m pytest tests/test_gpu_blocks.py tests/test_gpu_kernels.py -m gpu -v -rf -k 'relpos or probs or conv' --timeout 120 --timeout-method thread > gpurun_out/r06f_pytest.log 2>&1" \
  "for v in '' _a2; do for l in '' --legacy; do echo \"lib=\$v \$l\"; ESP_LIB_VARIANT=\$v timeout -k 10 120 python -u tools/attn_kernels_bench.py 256 --only probs \$l || exit 1; done; done > gpurun_out/r06f_probs.log 2>&1" \
  "timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_f_leg -o run -- python3 bench.py --rel-pos legacy --steps 5 --warmup 2 --no-cpu-baseline --feed-steps 0 > gpurun_out/prof_f_leg.log 2>&1" \
  "ESP_LIB_VARIANT=_a2 ESP_CONV2_BITS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_f_leg_a2 -o run -- python3 bench.py --rel-pos legacy --steps 5 --warmup 2 --no-cpu-baseline --feed-steps 0 > gpurun_out/prof_f_leg_a2.log 2>&1" \
  "timeout -k 10 300 python -u bench.py --no-cpu-baseline --feed-steps 0 --steps 20 > gpurun_out/r06f_bench.log 2>&1" \
  "timeout -k 10 300 python -u bench.py --rel-pos legacy --no-cpu-baseline --feed-steps 0 --steps 20 > gpurun_out/r06f_bench_legacy.log 2>&1"
