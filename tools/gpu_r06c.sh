#!/bin/bash
# round 6 (c): the attention block tests under the LDS slot-check build (relpos_probs_lds_kernel's slot
# generation words, esp_attn_slot_check_errors), then the B=128 bench fixture regenerated on the box's host
# (the oracle at B=128 needs ~130 GB: tests/golden/make_bench_fixture.py, now with whole-tensor fingerprints
# and the round-6 flip records), with a heartbeat so the long CPU run is not taken for a hang
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash gpurun_steps.sh \
  "ESP_LIB_VARIANT=_slotchk timeout -k 10 600 python -u -m pytest tests/test_gpu_blocks.py -m gpu -v -rf --timeout 300 --timeout-method thread > gpurun_out/r06c_pytest_slotchk.log 2>&1" \
  "(while true; do sleep 50; echo heartbeat \$(date +%T); done) & HB=\$!; timeout -k 10 1500 python -u tests/golden/make_bench_fixture.py gpurun_out/bench_c2_b128.npz > gpurun_out/r06c_bench_fixture.log 2>&1; rc=\$?; kill \$HB; exit \$rc"
