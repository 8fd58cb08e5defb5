#!/bin/bash
# Dev helper: one gpurun call, re-queued while the pod is busy (exit 3 /
# transient: nothing ran, nothing charged).  Usage: tools/gpu_run.sh TIMEOUT 'CMD'
T=$1; shift
for i in $(seq 1 60); do
  /usr/local/graft/bin/gpurun --timeout $T -- "$@"
  rc=$?
  st=$(python3 -c "import json;print(json.load(open('gpurun_out/.last_call.json'))['status'])" 2>/dev/null)
  if [ "$st" != "transient" ]; then exit $rc; fi
  echo "[gpu_run] transient ($st), retry in 90 s"; sleep 90
done
exit 3
