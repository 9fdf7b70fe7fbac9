#!/bin/bash
# round 6 (b): bench records -- C2 latest (the driver's line), C2 legacy (the SLURP YAML's rel-pos),
# the data-parallel path at N=1 (per-rank HBM of the N-GPU job) at B=256 and B=384, the C2 kernel trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/prof_b
bash gpurun_steps.sh \
  "timeout -k 10 600 python -u -m pytest tests/test_librispeech_config.py tests/test_gpu_model.py tests/test_gpu_graph.py -m gpu -v -s -rf --timeout 300 --timeout-method thread > gpurun_out/r06b_pytest_new.log 2>&1" \
  "timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/r06b_smoke.log 2>&1" \
  "timeout -k 10 400 python -u bench.py > gpurun_out/r06b_bench.log 2>&1" \
  "timeout -k 10 300 python -u bench.py --rel-pos legacy --no-cpu-baseline --feed-steps 0 > gpurun_out/r06b_bench_legacy.log 2>&1" \
  "timeout -k 10 300 python -u bench.py --dp-world1 --no-cpu-baseline --feed-steps 0 --steps 10 > gpurun_out/r06b_bench_dp_b256.log 2>&1" \
  "timeout -k 10 400 python -u bench.py --dp-world1 --batch 384 --no-cpu-baseline --feed-steps 0 --steps 10 > gpurun_out/r06b_bench_dp_b384.log 2>&1" \
  "timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_b -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --feed-steps 0 > gpurun_out/prof_b.log 2>&1"
