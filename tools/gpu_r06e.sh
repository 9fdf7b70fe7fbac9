#!/bin/bash
# round 6 (e): the DP tests and the DP path's HBM at N=1 after the capture's cache release; C5 (bf16) bench + kernel trace, the legacy C2 kernel trace, GEMM-family HBM traffic (two --pmc
# passes each) at C2 B=256 and C5 B=64
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/prof_e_c5 gpurun_out/prof_e_leg
bash gpurun_steps.sh \
  "timeout -k 10 600 python -u -m pytest tests/test_gpu_distributed.py tests/test_gpu_graph.py -m gpu -v -rf --timeout 300 --timeout-method thread > gpurun_out/r06e_pytest_dp.log 2>&1" \
  "timeout -k 10 300 python -u bench.py --dp-world1 --no-cpu-baseline --feed-steps 0 --steps 10 > gpurun_out/r06e_bench_dp_b256.log 2>&1" \
  "timeout -k 10 400 python -u bench.py --dp-world1 --batch 384 --no-cpu-baseline --feed-steps 0 --steps 10 > gpurun_out/r06e_bench_dp_b384.log 2>&1" \
  "timeout -k 10 300 python -u bench.py --config c5 --batch 64 --no-cpu-baseline --feed-steps 0 > gpurun_out/r06e_bench_c5_b64.log 2>&1" \
  "timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_e_c5 -o run -- python3 bench.py --config c5 --batch 64 --steps 5 --warmup 2 --no-cpu-baseline --feed-steps 0 > gpurun_out/prof_e_c5.log 2>&1" \
  "timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_e_leg -o run -- python3 bench.py --rel-pos legacy --steps 5 --warmup 2 --no-cpu-baseline --feed-steps 0 > gpurun_out/prof_e_leg.log 2>&1" \
  "bash tools/pmc_traffic.sh > gpurun_out/pmc_c2.log 2>&1" \
  "BENCH_ARGS='--config c5 --batch 64' TAG=c5 META='64 C5 512,12,1' bash tools/pmc_traffic.sh > gpurun_out/pmc_c5.log 2>&1"
