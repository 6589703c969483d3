#!/bin/bash
# One GPU call of round evidence: kernel timelines of the config stand-ins (tools/prof.sh trace),
# per-row numeric phase cycles of cant-like and wb-edu-like (tools/diag/v9 stamps build), and the
# bench command's rocprofv3 stats + FETCH/WRITE passes (tools/bench_profile.sh).
# usage: tools/round_evidence.sh <tag> "<matrices>" [stamps matrices]
set -o pipefail
tag=$1; mats=$2; smats=${3:-"cant wb-edu"}
out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp MHS_SYNTH_CACHE=/tmp/mhs_synth
bash tools/prof.sh $tag "$mats" trace > $out/prof.log 2>&1 || { tail -20 $out/prof.log; exit 1; }
grep -A30 "^== " $out/prof.log | grep -v "^--" | cut -c1-150
for m in $smats; do
  timeout -k 10 300 python3 -u tools/diag/stamps2.py $m > $out/stamps_$m.txt 2>&1 || { echo "stamps $m failed"; tail -5 $out/stamps_$m.txt; exit 1; }
  cat $out/stamps_$m.txt | tail -25
done
bash tools/bench_profile.sh $tag > $out/bench_profile.log 2>&1 || { tail -20 $out/bench_profile.log; exit 1; }
tail -5 $out/bench_profile.log
echo EVIDENCEDONE
