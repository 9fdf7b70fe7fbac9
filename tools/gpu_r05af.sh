#!/bin/bash
# round 5: peak HBM of the bench at B=256 / 384 (torch allocator peak reserved, graph pool included)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash gpurun_steps.sh \
  "timeout -k 10 400 python -u -c \"import runpy, sys, torch; sys.argv = ['bench.py', '--batch', '384', '--steps', '3', '--warmup', '2', '--no-cpu-baseline', '--feed-steps', '0']; runpy.run_path('bench.py', run_name='__main__'); print('PEAK_GiB B=384 reserved %.1f allocated %.1f' % (torch.cuda.max_memory_reserved() / 2**30, torch.cuda.max_memory_allocated() / 2**30))\" > gpurun_out/r05af_mem_b384.log 2>&1" \
  "timeout -k 10 400 python -u -c \"import runpy, sys, torch; sys.argv = ['bench.py', '--batch', '256', '--steps', '3', '--warmup', '2', '--no-cpu-baseline', '--feed-steps', '0']; runpy.run_path('bench.py', run_name='__main__'); print('PEAK_GiB B=256 reserved %.1f allocated %.1f' % (torch.cuda.max_memory_reserved() / 2**30, torch.cuda.max_memory_allocated() / 2**30))\" > gpurun_out/r05af_mem_b256.log 2>&1"
