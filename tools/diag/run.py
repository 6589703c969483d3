"""Time one ablation variant of the SpGEMM library on the cant-like workload.
usage: python tools/diag/run.py <variant-dir> [matrix]   (tools only; results of v!=0 are wrong by design)"""
import sys, json
from pathlib import Path
ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "mh-spgemm_amd")]
import numpy as np
import torch
import os
os.environ["MHS_LIB"] = str(Path(sys.argv[1]).resolve() / "libmhspgemm.so")
from mhspgemm import _lib
import mhspgemm
from mhspgemm import synth
name = sys.argv[2] if len(sys.argv) > 2 else "cant"
A = synth.SYNTH[name]()
A.H2D(0)
tool = mhspgemm.Tool(0)
ts = []
for i in range(25):
    C, t = mhspgemm.spgemm(tool, A, A)
    C.release()
    if i >= 5:
        ts.append(t)
med = lambda k: float(np.median([getattr(x, k) for x in ts]))
print(json.dumps({"variant": sys.argv[1], "Numeric": med("Numeric"), "Calculate_C_nnz": med("Calculate_C_nnz"),
                  "e2e": med("total_e2e")}))
