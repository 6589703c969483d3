#!/bin/bash
# The stamps build (with the probe guard) on cage15-like: does a lookup miss its table?
set -o pipefail
export TMPDIR=/tmp MHS_SYNTH_CACHE=/tmp/mhs_synth
out=gpurun_out/r05diag3; mkdir -p $out
python3 -c "import sys; sys.path[:0]=['.','mh-spgemm_amd']; from mhspgemm import synth; synth.load_or_synth('cage15')" > $out/synth.log 2>&1
STAMPS_LIB=ablib/stamps/libmhspgemm.so timeout -k 10 150 python3 -u tools/diag/stamps2.py cage15 > $out/stamps_cage15.txt 2>&1
echo "stamps rc=$?"
cat $out/stamps_cage15.txt | head -60
echo DIAG3DONE
