#!/bin/bash
# A/B: per-wave piece walks in the block kernels (MHS_NO_PIECES=1 variant as the base)
set -o pipefail
export TMPDIR=/tmp MHS_SYNTH_CACHE=/tmp/mhs_synth
out=gpurun_out/r05ab2; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -30 $out/pytest_gpu.log; exit 1; }
tail -1 $out/pytest_gpu.log
M="webbase-1M scircuit cant-s1 pdb1HYS cop20k_A mac_econ_fwd500 wb-edu"
for r in 1 2; do
  timeout -k 10 300 python tools/pipe.py $M --reps 3 --lib ablib/nopieces > $out/base_$r.jsonl 2>> $out/err.log || exit 1
  timeout -k 10 300 python tools/pipe.py $M --reps 3 > $out/new_$r.jsonl 2>> $out/err.log || exit 1
done
python3 tools/ab_pipe.py $out
echo AB2DONE
