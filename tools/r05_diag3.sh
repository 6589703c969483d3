#!/bin/bash
# (1) scircuit-like anatomy: kernel timelines with / without its hub rows and hub columns;
# (2) the stamps build (with the probe guard) on cage15-like: does a lookup miss its table?
set -o pipefail
export TMPDIR=/tmp MHS_SYNTH_CACHE=/tmp/mhs_synth
out=gpurun_out/r05diag3; mkdir -p $out
for v in both rows cols none; do
  timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $out/sc_$v -o run -- python3 tools/anatomy.py $v > $out/sc_$v.log 2>&1 || { echo "anatomy $v failed"; tail -5 $out/sc_$v.log; exit 1; }
  tail -1 $out/sc_$v.log
  python3 tools/timeline.py "$(find $out/sc_$v -name '*kernel_trace.csv' | head -1)" > $out/sc_$v.timeline 2>&1
  cat $out/sc_$v.timeline
done
python3 -c "import sys; sys.path[:0]=['.','mh-spgemm_amd']; from mhspgemm import synth; synth.load_or_synth('cage15')" > $out/synth.log 2>&1
STAMPS_LIB=ablib/stamps/libmhspgemm.so timeout -k 10 150 python3 -u tools/diag/stamps2.py cage15 > $out/stamps_cage15.txt 2>&1
echo "stamps rc=$?"
head -60 $out/stamps_cage15.txt
echo DIAG3DONE
