cd "${GRAFT_REPO_ROOT}"
rm -rf gpurun_out/prof
bash gpurun_steps.sh \
  "timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2>&1" \
  "timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof.log 2>&1"
