#!/bin/bash
# Kernel timelines of pipelined steps (tools/pipe.py under rocprofv3) + per-row numeric phase stamps
set -o pipefail
export TMPDIR=/tmp MHS_SYNTH_CACHE=/tmp/mhs_synth
out=gpurun_out/r05diag1; mkdir -p $out
for m in webbase-1M scircuit cop20k_A mac_econ_fwd500; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $out/$m -o run -- python3 tools/pipe.py $m --reps 1 --steps 10 > $out/$m.log 2>&1 || { echo "trace $m failed"; tail -5 $out/$m.log; exit 1; }
  python3 tools/timeline.py "$(find $out/$m -name '*kernel_trace.csv' | head -1)" > $out/$m/timeline.txt 2>&1
  echo "== $m"; cat $out/$m/timeline.txt
done
for m in webbase-1M scircuit; do
  STAMPS_LIB=ablib/stamps/libmhspgemm.so timeout -k 10 200 python3 -u tools/diag/stamps2.py $m > $out/stamps_$m.txt 2>&1 || { echo "stamps $m failed rc=$?"; tail -5 $out/stamps_$m.txt; exit 1; }
  tail -30 $out/stamps_$m.txt
done
STAMPS_LIB=ablib/stamps/libmhspgemm.so timeout -k 10 300 python3 -u tools/diag/stamps2.py cage15 > $out/stamps_cage15.txt 2>&1 || { echo "stamps cage15 failed rc=$?"; tail -8 $out/stamps_cage15.txt; exit 1; }
tail -30 $out/stamps_cage15.txt
echo DIAG1DONE
