#!/bin/bash
# Alternating A/B bench runs on one box: usage  bash tools/ab_bench.sh "<envA>" "<envB>" [rounds] [bench args]
# (env strings like "ESP_GEMM_ABL=64"; "-" for none).  Prints utt/s per run to gpurun_out/ab.log.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
A="$1"; B="$2"; R="${3:-2}"; shift 3; ARGS="$@"
[ "$A" = "-" ] && A=""; [ "$B" = "-" ] && B=""
mkdir -p gpurun_out
for i in $(seq 1 $R); do
  for which in A B; do
    if [ $which = A ]; then E="$A"; else E="$B"; fi
    out=$(env $E timeout -k 10 200 python bench.py --no-cpu-baseline --steps 15 --warmup 3 $ARGS 2>/dev/null | grep '^{') || exit 1
    v=$(echo "$out" | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])")
    echo "$which [$E] $v" | tee -a gpurun_out/ab.log
  done
done
