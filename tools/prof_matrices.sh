#!/bin/bash
# Kernel trace + stats of the sweep, one rocprofv3 run per matrix (gpurun_out/<tag>/<matrix>/).
# usage: tools/prof_matrices.sh <tag> matrix...
export TMPDIR=/tmp
tag=$1; shift
for m in "$@"; do
  out=gpurun_out/$tag/$m
  mkdir -p $out
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o run -- python3 tools/sweep.py $m --reps 5 > $out/log.txt 2>&1 || exit $?
  f=$(find $out -name '*kernel_stats.csv' | head -1)
  echo "== $m"; python3 tools/summarize_stats.py "$f"
done
