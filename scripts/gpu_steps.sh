#!/bin/bash
# Run GPU steps one after another, each under its own time limit; stop at the
# first step that dies abnormally (time limit, abort, segfault): a GPU fault
# must not be followed by more GPU work in the same call.  A plain test
# failure (pytest rc 1) does not stop later steps.
# usage: scripts/gpu_steps.sh "<seconds> <name> <command>" ...
mkdir -p gpurun_out
for step in "$@"; do
  secs=${step%% *}; rest=${step#* }; name=${rest%% *}; cmd=${rest#* }
  echo "[$(date +%T)] step $name: $cmd" | tee -a gpurun_out/steps.txt
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.txt" 2>&1
  rc=$?
  echo "[$(date +%T)] step $name rc=$rc" | tee -a gpurun_out/steps.txt
  tail -3 "gpurun_out/$name.txt"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
exit 0
