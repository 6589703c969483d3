"""Per-matrix sweep: median phase times, e2e GFLOPS and bin occupancy for every
BASELINE.json config matrix (synthetic stand-ins unless $MHS_MATRIX_DIR holds the
real files).  usage: python tools/sweep.py [matrix ...] [--lib DIR] [--reps N]"""
import argparse
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "mh-spgemm_amd")]
ap = argparse.ArgumentParser()
ap.add_argument("matrices", nargs="*", default=["cant", "webbase-1M", "mac_econ_fwd500", "scircuit", "cop20k_A", "cage15"])
ap.add_argument("--lib", default=None)
ap.add_argument("--reps", type=int, default=15)
ap.add_argument("--vendor", action="store_true", help="also time rocSPARSE (median of 3 after a warm-up)")
args = ap.parse_args()
if args.lib:
    os.environ["MHS_LIB"] = str(Path(args.lib).resolve() / "libmhspgemm.so")
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401
import mhspgemm  # noqa: E402
from mhspgemm import synth  # noqa: E402

keys = ["Form_mask_matrix_B", "symbolic_binning", "Calculate_C_nnz", "numeric_binning", "Numeric", "total_e2e"]
tool = mhspgemm.Tool(0)
for name in args.matrices:
    A, src = synth.load_or_synth(name)
    A.H2D(0)
    ts = []
    for i in range(args.reps + 3):
        C, t = mhspgemm.spgemm(tool, A, A)
        C.release()
        if i >= 3:
            ts.append(t)
    med = {k: round(float(np.median([getattr(x, k) for x in ts])), 4) for k in keys}
    flop = ts[-1].flop
    out = {"matrix": name, "src": src, "rows": A.M, "nnzA": A.nnz, "flop": int(flop), "nnzC": int(ts[-1].nnzC),
           "gflops_e2e": round(2 * flop / (med["total_e2e"] * 1e-3) / 1e9, 1), **med,
           "sym_bins": list(ts[-1].sym_bins), "num_bins": list(ts[-1].num_bins)}
    if args.vendor:
        vms = []
        for i in range(4):
            V, ms = mhspgemm.vendor_spgemm(tool, A, A)
            V.release()
            if i:
                vms.append(ms)
        out["rocsparse_ms"] = round(float(np.median(vms)), 4)
        out["rocsparse_gflops"] = round(2 * flop / (out["rocsparse_ms"] * 1e-3) / 1e9, 1)
        out["speedup_vs_rocsparse"] = round(out["rocsparse_ms"] / med["total_e2e"], 2)
    print(json.dumps(out), flush=True)
    A.d_release_csr()
    del A
tool.close()
