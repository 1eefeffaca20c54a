#!/bin/bash
# Local helper (never run on the GPU box): re-submit a gpurun call when no box was free.
# usage: tools/gpurun_slot_retry.sh <outfile> <timeout> '<command>'  -- retries ONLY when no box/slot was free (rc 3: nothing ran)
out=$1; to=$2; cmd=$3
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout $to -- "$cmd" > $out 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "status=transient" $out; then break; fi
  sleep 90
done
echo "done rc=$rc" >> $out
