cd "${GRAFT_REPO_ROOT}"
bash gpurun_steps.sh \
  "timeout -k 10 300 python -u bench.py --config c5 --batch 64 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_c5_b64.log 2>&1" \
  "timeout -k 10 300 python -u bench.py --config c4 --batch 64 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_c4_b64.log 2>&1" \
  "timeout -k 10 300 python -u bench.py --config c5 --batch 32 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_c5.log 2>&1"
