#!/bin/bash
# GPU suite on the recalibrated stand-ins; stamps (symbolic + numeric phases) of scircuit-,
# cop20k- and webbase-like; the default bench (verbose HBM shapes); then the stamps build without
# the numeric-body stamps on cage15-like (bisecting the stamps hang; last: it may not return)
set -o pipefail
export TMPDIR=/tmp MHS_SYNTH_CACHE=/tmp/mhs_synth
out=gpurun_out/r05diag4; mkdir -p $out
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -30 $out/pytest_gpu.log; exit 1; }
tail -1 $out/pytest_gpu.log
for m in scircuit cop20k_A webbase-1M; do
  STAMPS_LIB=ablib/stamps/libmhspgemm.so timeout -k 10 200 python3 -u tools/diag/stamps2.py $m > $out/stamps_$m.txt 2>&1 || { echo "stamps $m rc=$?"; tail -5 $out/stamps_$m.txt; exit 1; }
done
MHS_HBM_VERBOSE=1 timeout -k 10 500 python bench.py > $out/bench_default.json 2> $out/bench_default.err || { echo "bench failed"; tail $out/bench_default.err; exit 1; }
cut -c1-400 $out/bench_default.json; grep "hbm shape" $out/bench_default.err
python3 -c "import sys; sys.path[:0]=['.','mh-spgemm_amd']; from mhspgemm import synth; synth.load_or_synth('cage15')" > $out/synth.log 2>&1
STAMPS_LIB=ablib/stamps_nobody/libmhspgemm.so timeout -k 10 150 python3 -u tools/diag/stamps2.py cage15 > $out/stamps_nobody_cage15.txt 2>&1
echo "stamps_nobody cage15 rc=$?"
head -12 $out/stamps_nobody_cage15.txt
echo DIAG4DONE
