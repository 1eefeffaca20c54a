#!/bin/bash
# Run GPU steps in order; stop at the first step that did not exit 0/1
# (fault, abort, segfault, timeout) so nothing else touches the GPU after it.
# usage: tools/gpu_run.sh "<seconds> <logname> <cmd...>" ...
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for spec in "$@"; do
  secs=${spec%% *}; rest=${spec#* }; log=${rest%% *}; cmd=${rest#* }
  echo "=== [$log] $cmd (limit ${secs}s)" | tee -a gpurun_out/steps.log
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$log" 2>&1
  rc=$?
  echo "=== [$log] rc=$rc" | tee -a gpurun_out/steps.log
  tail -5 "gpurun_out/$log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
done
