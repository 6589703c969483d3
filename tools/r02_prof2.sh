#!/bin/bash
# kernel traces of the heavy matrices + SQ passes on cage15 + a sweep of every stand-in
export TMPDIR=/tmp MHS_SYNTH_CACHE=/tmp/mhs_synth
tag=${1:-r02g}; out=gpurun_out/$tag; mkdir -p $out
bash tools/prof_r02.sh $tag "webbase-1M cage15 wb-edu" trace || exit $?
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU" \
           "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_IDX_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $out/sq_$i -o run -- python3 tools/sweep.py cage15 --reps 1 > $out/sq_$i.log 2>&1 || { echo "sq pass $i failed rc=$?"; exit 1; }
done
echo "== sq done"
timeout -k 10 600 python tools/sweep.py cant cant-s1 cant-perturbed webbase-1M mac_econ_fwd500 scircuit cop20k_A cage15 pdb1HYS pwtk cage12 hood rma10 shipsec1 offshore wb-edu GAP-road delaunay_n24 --reps 5 --vendor > $out/sweep_all.jsonl 2> $out/sweep_all.err || { echo "sweep failed"; tail -5 $out/sweep_all.err; exit 1; }
echo R02PROF2DONE
