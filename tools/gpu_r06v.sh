#!/bin/bash
# round 6 (v): the fold epilogue with the row decomposition shared by both sub-tiles (default) vs its first form
# (_v0): c1fold alone (per-class trace) and its parity test, then alternating C2 B=384 bench lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/prof_v0 gpurun_out/prof_v1
bash gpurun_steps.sh \
  "timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -k 'c1fold or conv2_dgrad' --timeout 120 --timeout-method thread > gpurun_out/r06v_pytest.log 2>&1" \
  "ESP_LIB_VARIANT=_v0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_v0 -o run -- python3 tools/c1fold_bench.py > gpurun_out/r06v_c1fold_v0.log 2>&1" \
  "timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_v1 -o run -- python3 tools/c1fold_bench.py > gpurun_out/r06v_c1fold.log 2>&1" \
  "for v in _v0 '' _v0 ''; do echo \"lib=\$v\"; ESP_LIB_VARIANT=\$v timeout -k 10 400 python -u bench.py --no-cpu-baseline --feed-steps 0 --steps 20 | tail -1 || exit 1; done > gpurun_out/r06v_bench_ab.log 2>&1"
