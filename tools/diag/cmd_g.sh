export TMPDIR=/tmp; timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trw -o run -- python3 tools/diag/run_phases.py mh-spgemm_amd/mhspgemm webbase-1M > gpurun_out/trw.log 2>&1
timeout -k 10 300 python3 -c "
import sys; sys.path[:0]=['.','mh-spgemm_amd']
import torch, mhspgemm
from mhspgemm import synth
A = synth.SYNTH['webbase-1M'](); A.H2D(0)
t = mhspgemm.Tool(0)
C, tm = mhspgemm.spgemm(t, A, A)
print('sym', list(tm.sym_bins), 'num', list(tm.num_bins), 'nnzC', tm.nnzC)
" > gpurun_out/wbins.log 2>&1
