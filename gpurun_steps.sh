set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/sk_pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/sk_bench_bal_a.log 2>&1 &&
ESP_SPLITK_NOBALANCE=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/sk_bench_nobal_a.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/sk_bench_bal_b.log 2>&1 &&
ESP_SPLITK_NOBALANCE=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/sk_bench_nobal_b.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sk -o run -- python3 bench.py --steps 5 --warmup 3 > gpurun_out/sk_prof.log 2>&1
