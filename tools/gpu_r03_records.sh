#!/bin/bash
# Round-3 records: new tests, C2 / C5 bench lines, rocprofv3 kernel-trace summaries, GEMM-family
# HBM traffic (separate FETCH_SIZE / WRITE_SIZE passes) for C2 and C5, C5 per-shape GEMM rates.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/prof gpurun_out/prof_c5
bash gpurun_steps.sh \
 "timeout -k 10 200 python -u -m pytest tests/test_gpu_bf16.py -m gpu -x -v --timeout 150 --timeout-method thread -k 'loss_curve or amp_linear' > gpurun_out/pytest_new.log 2>&1" \
 "timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1" \
 "timeout -k 10 300 python bench.py --config c5 --batch 64 --no-cpu-baseline > gpurun_out/bench_c5.log 2>&1" \
 "timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof.log 2>&1" \
 "timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5 -o run -- python3 bench.py --config c5 --batch 64 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_c5.log 2>&1" \
 "timeout -k 10 200 python tools/gemm_profile.py --config c5 --batch 64 > gpurun_out/gemm_shapes_c5.log 2>&1" \
 "bash tools/pmc_traffic.sh" \
 "BENCH_ARGS='--config c5 --batch 64' TAG=c5 META='64 C5 512,12,1' bash tools/pmc_traffic.sh" || exit $?
python3 tools/prof_summary.py gpurun_out/prof 8 > gpurun_out/kernel_summary_c2.txt 2>&1
python3 tools/prof_summary.py gpurun_out/prof_c5 8 > gpurun_out/kernel_summary_c5.txt 2>&1
rm -rf gpurun_out/prof gpurun_out/prof_c5
