#!/bin/bash
# SQ counter passes (one rocprofv3 run per group of <= 4 SQ counters) on a bench command.
# usage: tools/prof_sq.sh <tag> <matrix>   -> gpurun_out/<tag>/sq_<i>/
export TMPDIR=/tmp
export MHS_SYNTH_CACHE=/tmp/mhs_synth
tag=$1
m=${2:-cant}
out=gpurun_out/$tag
mkdir -p $out
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU" \
           "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_IDX_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $out/sq_$i -o run -- python3 bench.py --matrix $m --steps 5 --warmup 1 --no-cpu > $out/sq_$i.log 2>&1 || { echo "sq pass $i ($grp) failed rc=$?"; exit 1; }
  echo "== sq pass $i done"
done
echo SQDONE
