#!/bin/bash
# HBM peak shapes (per-shape rates on stderr)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r05hbm; mkdir -p $out
timeout -k 10 200 python3 -c "
import sys, os; sys.path[:0]=['.','mh-spgemm_amd']; os.environ['MHS_HBM_VERBOSE']='1'
import mhspgemm; t=mhspgemm.Tool(0); print(t.hbm_peak(2<<30, 10)); t.close()" > $out/hbm.log 2>&1 || { tail -5 $out/hbm.log; exit 1; }
grep -v amdgpu $out/hbm.log
