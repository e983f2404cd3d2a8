#!/bin/bash
# Sequential GPU steps for one gpurun call: each step under its own time limit;
# stop at the first step that did not end normally (rc other than 0 / 1 = test
# failures), so a fault, abort or timeout never leads to another GPU step.
# usage: tools/gpu_run.sh "<seconds>|<name>|<command>" ...
set -u
mkdir -p gpurun_out
for spec in "$@"; do
  secs="${spec%%|*}"; rest="${spec#*|}"; name="${rest%%|*}"; cmd="${rest#*|}"
  echo "[gpu_run] $name: $cmd" | tee -a gpurun_out/gpu_run.log
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "[gpu_run] $name rc=$rc" | tee -a gpurun_out/gpu_run.log
  tail -3 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "[gpu_run] stopping after $name (rc=$rc)"; exit $rc; fi
done
