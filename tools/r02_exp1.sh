#!/bin/bash
export TMPDIR=/tmp MHS_SYNTH_CACHE=/tmp/mhs_synth
tag=r02c; out=gpurun_out/$tag; mkdir -p $out
for v in base g2048; do
  timeout -k 10 200 python tools/sweep.py cage15 cop20k_A --reps 5 --lib tools/var/$v > $out/sweep_$v.jsonl 2>$out/sweep_$v.err || { echo "sweep $v failed"; exit 1; }
  echo "== $v"; cat $out/sweep_$v.jsonl | cut -c1-400
  timeout -s KILL 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $out/fetch_$v -o run -- python3 tools/sweep.py cage15 --reps 1 --lib tools/var/$v > $out/fetch_$v.log 2>&1 || { echo "fetch $v failed"; exit 1; }
done
for m in cant webbase-1M cage15; do
  timeout -k 10 180 python tools/stamps.py $m > $out/stamps_$m.txt 2>&1 || { echo "stamps $m failed"; exit 1; }
  echo "== stamps $m"; cat $out/stamps_$m.txt
done
echo EXP1DONE
