#!/bin/bash
# GEMM-family HBM traffic at HEAD: two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) of one eager
# bench step, summarised on the box (the rocpd databases exceed what gpurun copies back).
# usage: [BENCH_ARGS="--config c5 --batch 64"] [TAG=c5] [META="64 C5 512,12,1"] bash tools/pmc_traffic.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
rm -rf gpurun_out/pmc_fetch gpurun_out/pmc_write
bash gpurun_steps.sh \
 "timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run -- python3 bench.py --eager --steps 1 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/pmc_fetch.log 2>&1" \
 "timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run -- python3 bench.py --eager --steps 1 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/pmc_write.log 2>&1" || exit $?
python3 tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write ${META:-256 C2 256,12,0} > gpurun_out/gemm_traffic${TAG:+_$TAG}.json 2>&1
rm -rf gpurun_out/pmc_fetch gpurun_out/pmc_write
