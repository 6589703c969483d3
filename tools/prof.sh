#!/bin/bash
# One parameterised profiling driver (replaces the per-round r0*_*.sh scripts).
#   tools/prof.sh <tag> "<matrices>" [modes]
# modes (comma list, default "trace"):
#   trace   rocprofv3 kernel trace + stats of tools/sweep.py (the product's own stream dealing)
#           and the timeline of the last full call -> <m>/timeline.txt
#   serial  the same with every numeric bin on one stream (MHS_NUM_STREAMS=1: per-kernel attribution)
#   pmc     FETCH_SIZE, WRITE_SIZE, TCC_HIT_sum+TCC_MISS_sum passes (one rocprofv3 run each,
#           numeric bins on one stream) -> <m>/pmc_<i>/
#   sweep   tools/sweep.py --reps 7 of all matrices -> sweep.jsonl
# Output under gpurun_out/<tag>/.  Every GPU step has its own time limit; the script stops
# at the first failure.
set -o pipefail
export TMPDIR=/tmp MHS_SYNTH_CACHE=/tmp/mhs_synth
tag=$1; mats=$2; modes=${3:-trace}
libarg=""; [ -n "$PROF_LIB" ] && libarg="--lib $PROF_LIB"  # PROF_LIB=<dir>: profile that library
out=gpurun_out/$tag; mkdir -p $out
has() { [[ ",$modes," == *",$1,"* ]]; }
csv() { find "$1" -name '*kernel_trace.csv' | head -1; }
if has sweep; then
  timeout -k 10 600 python3 tools/sweep.py $mats --reps 7 > $out/sweep.jsonl 2> $out/sweep.err || { tail -5 $out/sweep.err; exit 1; }
  cut -c1-200 $out/sweep.jsonl
fi
for m in $mats; do
  d=$out/$m; mkdir -p $d
  if has trace; then
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d/trace -o run -- python3 tools/sweep.py $m --reps 5 $libarg > $d/sweep.log 2>&1 || { echo "trace $m failed"; tail -5 $d/sweep.log; exit 1; }
    python3 tools/timeline.py "$(csv $d/trace)" > $d/timeline.txt 2>&1
    echo "== $m"; tail -1 $d/sweep.log | cut -c1-300; cat $d/timeline.txt
  fi
  if has serial; then
    MHS_NUM_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d/serial -o run -- python3 tools/sweep.py $m --reps 5 $libarg > $d/serial.log 2>&1 || { echo "serial $m failed"; exit 1; }
    python3 tools/timeline.py "$(csv $d/serial)" > $d/timeline_serial.txt 2>&1
    echo "== $m (one stream)"; cat $d/timeline_serial.txt
  fi
  if has pmc; then
    i=0
    for g in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
      i=$((i+1))
      MHS_NUM_STREAMS=1 timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $g --output-format csv -d $d/pmc_$i -o run -- python3 tools/sweep.py $m --reps 2 $libarg > $d/pmc_$i.log 2>&1 || { echo "pmc $g $m failed"; exit 1; }
      echo "== $m pmc $g ok"
    done
  fi
done
echo ALLDONE
