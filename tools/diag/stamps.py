"""Per-phase cycle breakdown of numeric rows (diag build 9): s_memtime deltas per row and phase."""
import sys, ctypes, os
from pathlib import Path
ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "mh-spgemm_amd")]
os.environ["MHS_LIB"] = str(ROOT / "tools/diag/v9/libmhspgemm.so")
import numpy as np, torch
from mhspgemm import _lib
import mhspgemm
from mhspgemm import synth
A = synth.SYNTH[sys.argv[1] if len(sys.argv) > 1 else "cant"](); A.H2D(0)
tool = mhspgemm.Tool(0)
L = _lib.lib(); L.mhs_diag_setup.argtypes = [ctypes.c_int, ctypes.c_void_p]
dev = ctypes.c_void_p()
assert L.mhs_diag_setup(A.M, ctypes.byref(dev)) == 0
for i in range(3):
    C, t = mhspgemm.spgemm(tool, A, A); C.release()
buf = np.zeros(A.M * 8, np.uint64)
L.mhs_memcpy(tool.ctx, buf.ctypes.data, dev, buf.nbytes, 1)
ph = buf.reshape(A.M, 8).astype(np.float64)
names = ["prologue", "tiles(load/build)", "bases(+rmap)", "clear_acc", "accumulate", "output"]
tot = ph[:, :6].sum()
for k, nm in enumerate(names):
    print(f"{nm:20s} {ph[:, k].mean():10.0f} cycles/row (median {np.median(ph[:, k]):8.0f})  {100*ph[:, k].sum()/tot:5.1f}%")
print("Numeric ms", t.Numeric, "Calculate_C_nnz ms", t.Calculate_C_nnz)
