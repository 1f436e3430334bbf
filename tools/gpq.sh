#!/bin/bash
# usage: gpq.sh OUTFILE TIMEOUT 'command'   -- retries only while no slot/box is free (rc 3)
out=$1; to=$2; cmd=$3
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout $to -- "$cmd" > $out 2>&1; rc=$?
  if [ $rc -ne 3 ] && ! grep -q "retry in a few minutes" $out; then break; fi
  sleep 90
done
echo "GPQ_DONE rc=$rc tries=$i" >> $out
