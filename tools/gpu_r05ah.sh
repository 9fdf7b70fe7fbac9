#!/bin/bash
# round 5: s_setprio 1 around each k-step's MFMAs (ESP_GEMM_SETPRIO=1, libespnet_mi355_sp.so) vs none: GEMM parity
# under the variant, GEMM timings, bench A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=gpurun_out/r05ah_gemm.txt
rm -f $T
bash gpurun_steps.sh \
  "ESP_LIB_VARIANT=_sp timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k 'gemm or planes or relpos_dqv or conv2' -x -q --timeout 120 --timeout-method thread > gpurun_out/r05ah_pytest_sp.log 2>&1" \
  "for v in '' _sp; do for s in '1 1 1024 256 95744 20 --rowsum' '1 1 256 256 95744 20 --rowsum' '0 1 95744 256 1024 20 --bw' '0 0 95744 1024 256 20 --bw' '0 0 95744 1024 256 20'; do ESP_LIB_VARIANT=\$v timeout -k 10 60 python -u tools/gemm_one.py \$s >> $T 2>&1 || exit 1; echo \"  [\$v] \$s\" >> $T; done; done" \
  "timeout -k 10 400 python -u bench.py --no-cpu-baseline --feed-steps 0 > gpurun_out/r05ah_bench.log 2>&1" \
  "ESP_LIB_VARIANT=_sp timeout -k 10 400 python -u bench.py --no-cpu-baseline --feed-steps 0 > gpurun_out/r05ah_bench_sp.log 2>&1" \
  "timeout -k 10 400 python -u bench.py --no-cpu-baseline --feed-steps 0 > gpurun_out/r05ah_bench2.log 2>&1" \
  "ESP_LIB_VARIANT=_sp timeout -k 10 400 python -u bench.py --no-cpu-baseline --feed-steps 0 > gpurun_out/r05ah_bench_sp2.log 2>&1"
