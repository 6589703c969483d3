#!/bin/bash
# Kernel timelines (last full pipelined step) of the small configs after the scattered class
set -o pipefail
export TMPDIR=/tmp MHS_SYNTH_CACHE=/tmp/mhs_synth
out=gpurun_out/r05diag6; mkdir -p $out
for m in scircuit mac_econ_fwd500 cop20k_A webbase-1M; do
  timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $out/$m -o run -- python3 tools/pipe.py $m --reps 1 --steps 10 > $out/$m.log 2>&1 || { echo "$m failed"; tail -5 $out/$m.log; exit 1; }
  python3 tools/timeline.py "$(find $out/$m -name '*kernel_trace.csv' | head -1)" > $out/$m.timeline 2>&1
  echo "== $m"; cat $out/$m.timeline
done
echo DIAG6DONE
