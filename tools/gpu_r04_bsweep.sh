cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
bash gpurun_steps.sh \
  "timeout -k 10 300 python -u bench.py --batch 128 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bs128.log 2>&1" \
  "timeout -k 10 300 python -u bench.py --batch 192 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bs192.log 2>&1" \
  "timeout -k 10 300 python -u bench.py --batch 256 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bs256.log 2>&1"
