"""Median per-phase times (timing=True calls) of one library variant.
usage: python tools/diag/run_phases.py <variant-dir> [matrix]"""
import sys, json, os
from pathlib import Path
ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "mh-spgemm_amd")]
import numpy as np
import torch
os.environ["MHS_LIB"] = str(Path(sys.argv[1]).resolve() / "libmhspgemm.so")
import mhspgemm
from mhspgemm import synth
A = synth.SYNTH[sys.argv[2] if len(sys.argv) > 2 else "cant"]()
A.H2D(0)
tool = mhspgemm.Tool(0)
ts = []
for i in range(25):
    C, t = mhspgemm.spgemm(tool, A, A)
    C.release()
    if i >= 5:
        ts.append(t)
keys = ["Form_mask_matrix_B", "symbolic_binning", "Calculate_C_nnz", "numeric_binning", "Numeric", "total_e2e"]
print(json.dumps({k: round(float(np.median([getattr(x, k) for x in ts])), 4) for k in keys}))
