#!/bin/bash
# Round-2 evidence on one GPU box, written under gpurun_out/<tag>/:
#   avail.txt                  rocprofv3 -L (counter names of this box)
#   <matrix>/                  kernel trace + stats of tools/sweep.py <matrix> (timeline per call)
#   <matrix>/fetch|write       FETCH_SIZE / WRITE_SIZE passes of the same command (separate runs)
#   sq_<k>/                    SQ counter passes of the cant bench (one pass per group)
# usage: tools/prof_r02.sh <tag> "<matrices>" [pmc]  -- every step under its own time limit,
# the chain stops at the first failure.
export TMPDIR=/tmp
export MHS_SYNTH_CACHE=/tmp/mhs_synth
tag=$1
mats=$2
what=${3:-trace}
out=gpurun_out/$tag
mkdir -p $out
if [ ! -f $out/avail.txt ]; then
  timeout -s KILL 60 rocprofv3 -L > $out/avail.txt 2>&1 || echo "rocprofv3 -L rc=$?"
fi
for m in $mats; do
  d=$out/$m
  mkdir -p $d
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d/trace -o run -- python3 tools/sweep.py $m --reps 5 > $d/sweep.log 2>&1 || { echo "trace $m failed"; exit 1; }
  echo "== $m trace done"; tail -1 $d/sweep.log
  if [ "$what" = "pmc" ]; then
    timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $d/fetch -o run -- python3 tools/sweep.py $m --reps 2 > $d/fetch.log 2>&1 || { echo "fetch $m failed"; exit 1; }
    timeout -s KILL 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $d/write -o run -- python3 tools/sweep.py $m --reps 2 > $d/write.log 2>&1 || { echo "write $m failed"; exit 1; }
    echo "== $m pmc done"
  fi
done
echo ALLDONE
