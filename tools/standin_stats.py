"""Statistics of synthetic stand-ins (M, nnz(A), flop, nnz(C) by the oracle, longest row) in the
form of mhspgemm.synth.ACHIEVED.  usage: python tools/standin_stats.py cage15 scircuit ..."""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / 'mh-spgemm_amd')]
import numpy as np
from mhspgemm import synth
from oracle import oracle as orc
import mhspgemm
for name in sys.argv[1:]:
    A = synth.SYNTH[name]()
    f = mhspgemm.flop_count_np(A.col, A.ptr)
    Cp, Ci, Cv = orc.spgemm(A.ptr, A.col, A.val, A.ptr, A.col, A.val, A.N)
    print(f'    "{name}": dict(M={A.M:_}, nnzA={A.nnz:_}, flop={f:_}, nnzC={int(Cp[-1]):_}, max_row={int(np.diff(A.ptr).max())}),', flush=True)
    del Cp, Ci, Cv
