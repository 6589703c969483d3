#!/bin/bash
# Chained GPU steps for one gpurun call.  Each step has its own time limit.
# Continue after a step only if it ended normally (rc 0, or 1 = test failures);
# stop on crashes / aborts / timeouts (134, 139, 124, 137, ...).
# usage: tools/gpu_run.sh <tag> "<cmd1>" "<cmd2>" ...   (each cmd: "<seconds>|<command>")
tag=$1; shift
mkdir -p gpurun_out
i=0
for spec in "$@"; do
  i=$((i+1))
  lim=${spec%%|*}; cmd=${spec#*|}
  log=gpurun_out/${tag}_step${i}.log
  echo "=== step $i (limit ${lim}s): $cmd" | tee -a gpurun_out/${tag}_summary.log
  timeout -k 10 "$lim" bash -c "$cmd" > "$log" 2>&1
  rc=$?
  echo "=== step $i rc=$rc" | tee -a gpurun_out/${tag}_summary.log
  tail -25 "$log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: step $i rc=$rc"; exit $rc; fi
done
