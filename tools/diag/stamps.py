"""Per-phase cycle breakdown of the numeric rows (diag build 9)."""
import sys, ctypes
from pathlib import Path
ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "mh-spgemm_amd")]
import numpy as np, torch
import os
os.environ["MHS_LIB"] = str(ROOT / "tools/diag/v9/libmhspgemm.so")
from mhspgemm import _lib
import mhspgemm
from mhspgemm import synth
A = synth.SYNTH[sys.argv[1] if len(sys.argv) > 1 else "cant"](); A.H2D(0)
tool = mhspgemm.Tool(0)
L = _lib.lib(); L.mhs_diag_read.argtypes = [ctypes.c_void_p]
buf = np.zeros(8, np.uint64)
for i in range(3):
    C, t = mhspgemm.spgemm(tool, A, A); C.release()
L.mhs_diag_read(buf.ctypes.data)
names = ["prologue", "clear+build_tiles", "scan_bases", "clear_acc", "accumulate", "output"]
tot = buf[:6].sum()
for k, nm in enumerate(names):
    print(f"{nm:20s} {buf[k]/3/A.M:12.0f} cycles/row  {100*buf[k]/tot:5.1f}%")
print("Numeric ms", t.Numeric)
