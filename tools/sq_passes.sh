#!/bin/bash
# SQ counters of the bench command's kernels (4 passes of <= 4 SQ counters each, one rocprofv3
# run a pass) for the given matrices -> gpurun_out/<tag>/<matrix>/pmc_<i>/ ; summarised by
# tools/sq_summary.py.   usage: tools/sq_passes.sh <tag> "<matrices>"
set -o pipefail
export TMPDIR=/tmp MHS_SYNTH_CACHE=/tmp/mhs_synth
tag=$1; mats=$2; out=gpurun_out/$tag
passes=("SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU"
        "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_IDX_ACTIVE")
for m in $mats; do
  i=0
  for p in "${passes[@]}"; do
    i=$((i+1)); d=$out/$m/pmc_$i; mkdir -p $d
    timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $p --output-format csv -d $d -o run -- python3 bench.py --matrix $m --no-cpu --no-configs > $d.log 2>&1 || { echo "pass $i $m failed"; tail -3 $d.log; exit 1; }
    echo "== $m pass $i ok"
  done
done
echo SQDONE
