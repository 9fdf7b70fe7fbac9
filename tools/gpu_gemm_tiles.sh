cd "${GRAFT_REPO_ROOT}"
export GEMM_BENCH_B=128
bash gpurun_steps.sh \
 "timeout -k 10 200 python -u tools/gemm_bench.py > gpurun_out/gemm_default.log 2>&1" \
 "ESP_GEMM_BNT=128 timeout -k 10 200 python -u tools/gemm_bench.py 4 5 6 14 > gpurun_out/gemm_bnt128.log 2>&1" \
 "ESP_GEMM_BNT=64 timeout -k 10 200 python -u tools/gemm_bench.py 0 1 2 3 7 15 16 > gpurun_out/gemm_bnt64.log 2>&1"
