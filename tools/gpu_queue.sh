#!/bin/bash
# queue a gpurun call: retry ONLY while the pool reports no free box/slot (status "transient": nothing ran, nothing charged)
# usage: q.sh TIMEOUT 'command' LOG
T="$1"; CMD="$2"; LOG="$3"
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  st=$(python3 -c "import json;print(json.load(open('/root/repo/gpurun_out/.last_call.json')).get('status',''))" 2>/dev/null)
  if [ "$st" != "transient" ]; then echo "rc=$rc status=$st attempt=$i" >> "$LOG"; exit $rc; fi
  sleep 90
done
echo "gave up" >> "$LOG"
