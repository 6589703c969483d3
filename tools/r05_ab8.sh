#!/bin/bash
# A/B: the rare symbolic bins forked onto an aux stream for every call (MHS_SYM_FORK=1) vs the
# default (fork from 512 K rows, or numeric-first with rows past the tiny classes)
set -o pipefail
export TMPDIR=/tmp MHS_SYNTH_CACHE=/tmp/mhs_synth
out=gpurun_out/r05ab8; mkdir -p $out
M="scircuit cop20k_A webbase-1M mac_econ_fwd500 cant cant-s1 offshore cage15"
for r in 1 2; do
  timeout -k 10 400 python tools/pipe.py $M --reps 3 > $out/base_$r.jsonl 2>> $out/err.log || { tail -5 $out/err.log; exit 1; }
  MHS_SYM_FORK=1 timeout -k 10 400 python tools/pipe.py $M --reps 3 > $out/fork_$r.jsonl 2>> $out/err.log || { tail -5 $out/err.log; exit 1; }
done
python3 tools/ab_pipe.py $out
echo AB8DONE
