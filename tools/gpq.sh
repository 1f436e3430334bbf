#!/bin/bash
# usage: gpq.sh OUTFILE TIMEOUT 'command'   -- retries only while no slot/box is free (rc 3)
# Each attempt's output is appended to OUTFILE (the last attempt's verdict is at its end).
out=$1; to=$2; cmd=$3
: > $out
for i in $(seq 1 60); do
  echo "=== attempt $i $(date +%T)" >> $out
  /usr/local/graft/bin/gpurun --timeout $to -- "$cmd" > $out.tmp 2>&1; rc=$?
  grep -v "every call sends the whole tree" $out.tmp >> $out
  if [ $rc -ne 3 ] && ! grep -q "retry in" $out.tmp; then break; fi
  sleep 90
done
rm -f $out.tmp
echo "GPQ_DONE rc=$rc tries=$i" >> $out
