#!/bin/bash
# gpurun wrapper: retries ONLY when gpurun reports an infrastructure-side transient failure
# before anything ran (status=transient, run_s=0). Any real run result is returned as is.
for attempt in 1 2 3 4; do
  /usr/local/graft/bin/gpurun "$@"
  rc=$?
  st=$(python3 -c "import json;d=json.load(open('gpurun_out/.last_call.json'));print(d['status'], d.get('run_s') or 0)" 2>/dev/null)
  set -- "$@"
  if [[ "$st" == transient* ]] && [[ "$st" == *" 0"* || "$st" == *" 0.0"* || "$st" == *"None"* ]]; then
    echo "[gpu.sh] transient infrastructure failure before run; retry $attempt after 45s"
    sleep 45
    continue
  fi
  exit $rc
done
exit $rc
