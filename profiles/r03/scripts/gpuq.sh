#!/bin/bash
# Submit one gpurun command; when the pod has no free slot or the box was lost before anything
# ran (status "transient", nothing charged) wait and submit the same command again, up to 12
# times.  Any run that actually started is never repeated.
# usage: tools/r03/gpuq.sh <timeout_s> '<command>' <log>
T=$1; CMD=$2; LOG=$3
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$CMD" > "$LOG" 2>&1
  st=$(python3 -c "import json; print(json.load(open('/root/repo/gpurun_out/.last_call.json')).get('status'))" 2>/dev/null)
  if [ "$st" != "transient" ]; then echo "status=$st attempt=$i" >> "$LOG"; exit 0; fi
  sleep 120
done
echo "gave up after 12 transient attempts" >> "$LOG"
