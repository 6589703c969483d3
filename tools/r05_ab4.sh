#!/bin/bash
# A/B: first A chunk prefetched before the tile table in single wave rows (MHS_PRE_CHUNK), at the
# 8-wave (spills) and 7-wave register budgets of the 5 KiB hash kernel; GPU suite on the new default
set -o pipefail
export TMPDIR=/tmp MHS_SYNTH_CACHE=/tmp/mhs_synth
out=gpurun_out/r05ab4; mkdir -p $out
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -30 $out/pytest_gpu.log; exit 1; }
tail -1 $out/pytest_gpu.log
M="cop20k_A webbase-1M scircuit mac_econ_fwd500 cage12 offshore cage15"
for r in 1 2; do
  for v in nopre pre8 pre7; do
    lib=""; [ $v != pre8 ] && lib="--lib ablib/$v"
    timeout -k 10 400 python tools/pipe.py $M --reps 3 $lib > $out/${v}_$r.jsonl 2>> $out/err.log || { tail -5 $out/err.log; exit 1; }
  done
done
python3 tools/ab_pipe.py $out
echo AB4DONE
