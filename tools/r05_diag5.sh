#!/bin/bash
# SQ counters of cop20k- and webbase-like's kernels (4 passes each) + the HBM peak shapes
set -o pipefail
export TMPDIR=/tmp MHS_SYNTH_CACHE=/tmp/mhs_synth
out=gpurun_out/r05diag5; mkdir -p $out
bash tools/sq_passes.sh r05diag5 "cop20k_A webbase-1M" > $out/sq.log 2>&1 || { tail -5 $out/sq.log; exit 1; }
for m in cop20k_A webbase-1M; do python3 tools/sq_summary.py r05diag5 $m $out/$m; done
timeout -k 10 200 python3 -c "
import sys, os; sys.path[:0]=['.','mh-spgemm_amd']; os.environ['MHS_HBM_VERBOSE']='1'
import mhspgemm; t=mhspgemm.Tool(0); print(t.hbm_peak(2<<30, 10)); t.close()" > $out/hbm.log 2>&1 || { tail -5 $out/hbm.log; exit 1; }
cat $out/hbm.log | grep -v amdgpu
echo DIAG5DONE
