#!/bin/bash
# Alternating bench runs over several env settings on one box:
#   bash tools/abc_bench.sh <rounds> "<env1>" "<env2>" ... [-- bench args]   ("-" = no env)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$1"; shift
ENVS=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do ENVS+=("$1"); shift; done
[ "$1" = "--" ] && shift
ARGS="$@"
mkdir -p gpurun_out
for i in $(seq 1 $R); do
  for E in "${ENVS[@]}"; do
    [ "$E" = "-" ] && E=""
    out=$(env $E timeout -k 10 200 python bench.py --no-cpu-baseline --steps 15 --warmup 3 $ARGS 2>/dev/null | grep '^{') || exit 1
    v=$(echo "$out" | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])")
    echo "[$E] $v" | tee -a gpurun_out/abc.log
  done
done
