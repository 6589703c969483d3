#!/bin/bash
# Round-2 profile call 1: kernel traces + FETCH/WRITE passes of the six config matrices,
# SQ counter passes on the cant bench, per-phase stamps (diag build) of three matrices.
export TMPDIR=/tmp MHS_SYNTH_CACHE=/tmp/mhs_synth
tag=${1:-r02b}
mkdir -p gpurun_out/$tag
bash tools/prof_r02.sh $tag "cant webbase-1M mac_econ_fwd500 scircuit cop20k_A cage15" pmc || exit $?
bash tools/prof_sq.sh $tag cant || exit $?
for m in cant webbase-1M cage15; do
  timeout -k 10 180 python tools/stamps.py $m > gpurun_out/$tag/stamps_$m.txt 2>&1 || { echo "stamps $m failed"; exit 1; }
  echo "== stamps $m"; cat gpurun_out/$tag/stamps_$m.txt
done
echo R02PROF1DONE
