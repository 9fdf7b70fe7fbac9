set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ESP_GEMM_ABL=32 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/nt2_bench_nt_a.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/nt2_bench_default_a.log 2>&1 &&
ESP_GEMM_ABL=32 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/nt2_bench_nt_b.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/nt2_bench_default_b.log 2>&1 &&
ESP_GEMM_ABL=32 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_nt -o run -- python3 bench.py --steps 5 --warmup 3 > gpurun_out/nt2_prof_nt.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_def -o run -- python3 bench.py --steps 5 --warmup 3 > gpurun_out/nt2_prof_def.log 2>&1
