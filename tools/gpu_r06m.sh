#!/bin/bash
# round 6 (m): conv1's bit map staged in LDS and written coalesced per block -- conv1 microbench against the
# previous build (_c0), the full GPU suite, a bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash gpurun_steps.sh \
  "for v in _c0 '' _c0 ''; do echo \"lib=\$v\"; ESP_LIB_VARIANT=\$v timeout -k 10 150 python -u tools/conv1_bench.py || exit 1; done > gpurun_out/r06m_conv1.log 2>&1" \
  "timeout -k 10 1100 python -u -m pytest tests -m gpu -v -rf --timeout 350 --timeout-method thread > gpurun_out/r06m_pytest_gpu.log 2>&1" \
  "for v in _c0 '' _c0 ''; do echo \"lib=\$v\"; ESP_LIB_VARIANT=\$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --feed-steps 0 --steps 20 | tail -1 || exit 1; done > gpurun_out/r06m_bench_ab.log 2>&1"
