#!/bin/bash
# gpurun with waits while the pool has no free box (status "transient": nothing ran, nothing charged)
LOG=$1; shift
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun "$@" > "$LOG" 2>&1
  st=$(python3 -c "import json;print(json.load(open('gpurun_out/.last_call.json'))['status'])" 2>/dev/null)
  if grep -q "status=transient" "$LOG"; then sleep 90; continue; fi
  break
done
tail -45 "$LOG"
