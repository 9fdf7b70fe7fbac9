set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_flash.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r02h_flash_tests.log 2>&1 &&
timeout -k 10 300 python -u tools/flash_bench.py 128 > gpurun_out/r02h_flash_bench.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA -d gpurun_out/pmc1_r02h -o run -- python3 tools/flash_bench.py 128 > gpurun_out/r02h_pmc1.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU -d gpurun_out/pmc2_r02h -o run -- python3 tools/flash_bench.py 128 > gpurun_out/r02h_pmc2.log 2>&1
