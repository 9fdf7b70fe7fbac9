set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r02d_bench_head.log 2>&1 &&
timeout -k 10 300 python -u tools/gemm_profile.py --batch 128 > gpurun_out/r02d_gemm_shapes.txt 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r02d -o run -- python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline > gpurun_out/r02d_prof.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_r02d -o run -- python3 bench.py --eager --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r02d_pmc_fetch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_r02d -o run -- python3 bench.py --eager --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r02d_pmc_write.log 2>&1
