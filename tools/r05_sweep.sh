#!/bin/bash
# Round-5 sweep of every stand-in (16matrix.txt + the cant variants): synchronised calls with
# per-phase events, median of 5, rocSPARSE beside it -> gpurun_out/<tag>/sweep_all.jsonl
set -o pipefail
export TMPDIR=/tmp MHS_SYNTH_CACHE=/tmp/mhs_synth
tag=$1; out=gpurun_out/$tag; mkdir -p $out
M="cant cant-s1 cant-perturbed webbase-1M mac_econ_fwd500 scircuit cop20k_A cage15 pdb1HYS pwtk cage12 hood rma10 shipsec1 offshore wb-edu GAP-road delaunay_n24"
for m in $M; do
  timeout -k 10 300 python3 tools/sweep.py $m --reps 5 --vendor >> $out/sweep_all.jsonl 2>> $out/sweep.err || { echo "$m failed"; tail -5 $out/sweep.err; exit 1; }
  echo "$m done"
done
python3 tools/baseline_table.py $out/sweep_all.jsonl
echo SWEEPDONE
