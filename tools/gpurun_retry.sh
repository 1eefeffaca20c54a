#!/bin/bash
# Host-side wrapper: re-submit a gpurun call only when the GPU service
# reports an infrastructure event (box lost while being prepared, backoff,
# no slot) — never after the command itself ran.
# usage: tools/gpurun_retry.sh <timeout> '<command>'
t=$1; shift
for attempt in 1 2 3 4 5 6; do
  out=$(/usr/local/graft/bin/gpurun --timeout "$t" -- "$@" 2>&1); rc=$?
  if echo "$out" | grep -q "run 0.0s of limit\|backing off\|run Nones\|no box\|slot free"; then
    echo "[retry $attempt] infrastructure: $(echo "$out" | grep '^\[gpurun\]' | tail -1)"; sleep 45; continue
  fi
  echo "$out" | grep -v "^\[gpurun\] sending" | tail -8; exit $rc
done
echo "gave up after 6 infrastructure failures"; exit 3
