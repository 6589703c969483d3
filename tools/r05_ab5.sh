#!/bin/bash
# A/B: row-cache / spill list entries loaded before the table clear and a few at a time (head =
# the previous commit's library); GPU suite on the new default
set -o pipefail
export TMPDIR=/tmp MHS_SYNTH_CACHE=/tmp/mhs_synth
out=gpurun_out/r05ab5; mkdir -p $out
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -30 $out/pytest_gpu.log; exit 1; }
tail -1 $out/pytest_gpu.log
M="scircuit cop20k_A webbase-1M mac_econ_fwd500 cant cant-s1 offshore cage15"
for r in 1 2; do
  for v in head new; do
    lib=""; [ $v != new ] && lib="--lib ablib/$v"
    timeout -k 10 400 python tools/pipe.py $M --reps 3 $lib > $out/${v}_$r.jsonl 2>> $out/err.log || { tail -5 $out/err.log; exit 1; }
  done
done
python3 tools/ab_pipe.py $out
echo AB5DONE
