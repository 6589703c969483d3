#!/bin/bash
# GPU suite (new path-counter tests), then the stamps build on cage15-like with every kernel
# serialised and HIP's API log: the last launch in the log is the one that does not finish.
set -o pipefail
export TMPDIR=/tmp MHS_SYNTH_CACHE=/tmp/mhs_synth
out=gpurun_out/r05diag2; mkdir -p $out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -30 $out/pytest_gpu.log; exit 1; }
tail -1 $out/pytest_gpu.log
python3 -c "import sys; sys.path[:0]=['.','mh-spgemm_amd']; from mhspgemm import synth; synth.load_or_synth('cage15')" > $out/synth.log 2>&1
STAMPS_LIB=ablib/stamps/libmhspgemm.so AMD_SERIALIZE_KERNEL=3 AMD_LOG_LEVEL=4 timeout -k 10 150 python3 -u tools/diag/stamps2.py cage15 > $out/stamps_cage15.txt 2> $out/stamps_cage15.err
rc=$?
echo "stamps rc=$rc"
tail -5 $out/stamps_cage15.txt
grep -a "ShaderName" $out/stamps_cage15.err | tail -6
echo DIAG2DONE
