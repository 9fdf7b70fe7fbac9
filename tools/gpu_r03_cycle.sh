rm -rf gpurun_out/prof gpurun_out/pmc_a1 gpurun_out/pmc_a2
bash gpurun_steps.sh \
 "timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_bf16.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gemm.log 2>&1" \
 "timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1" \
 "timeout -k 10 200 python bench.py > gpurun_out/bench.log 2>&1" \
 "timeout -k 10 200 python tools/gemm_profile.py --batch 128 > gpurun_out/gemm_shapes.log 2>&1" \
 "timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof.log 2>&1" \
 "timeout -k 10 200 python tools/gemm_profile.py --config c5 --batch 64 > gpurun_out/gemm_shapes_c5.log 2>&1" \
 "timeout -k 10 120 python3 tools/attn_kernels_bench.py 128 > gpurun_out/attn_k.log 2>&1" \
 "timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA -d gpurun_out/pmc_a1 -o run -- python3 tools/attn_kernels_bench.py 128 > gpurun_out/pmc_a1.log 2>&1" \
 "timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_INSTS_SALU -d gpurun_out/pmc_a2 -o run -- python3 tools/attn_kernels_bench.py 128 > gpurun_out/pmc_a2.log 2>&1"
