"""Per-phase cycle totals of numeric rows (MHS_ROW_STAMPS build in tools/diag/v9), heads
only.  usage: python tools/diag/stamps2.py <matrix>   (prints progress: long runs stay visible)"""
import sys, ctypes, os, time
from pathlib import Path
ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "mh-spgemm_amd")]
os.environ["MHS_LIB"] = os.environ.get("STAMPS_LIB", str(ROOT / "tools/diag/v9/libmhspgemm.so"))
import numpy as np, torch
from mhspgemm import _lib
import mhspgemm
from mhspgemm import synth
t0 = time.time()
name = sys.argv[1] if len(sys.argv) > 1 else "cant"
A, _ = synth.load_or_synth(name)
print(f"[{time.time()-t0:.1f}s] matrix {name} rows {A.M}", flush=True)
A.H2D(0)
tool = mhspgemm.Tool(0)
L = _lib.lib(); L.mhs_diag_setup.argtypes = [ctypes.c_int, ctypes.c_void_p]
dev = ctypes.c_void_p()
assert L.mhs_diag_setup(A.M, ctypes.byref(dev)) == 0
sdev = ctypes.c_void_p()
if hasattr(L, "mhs_diag_setup_sym"):  # symbolic rows' phases (sym_row_s)
    L.mhs_diag_setup_sym.argtypes = [ctypes.c_int, ctypes.c_void_p]
    assert L.mhs_diag_setup_sym(A.M, ctypes.byref(sdev)) == 0
g = (ctypes.c_ulonglong * 8)()
for i in range(3):
    C, t = mhspgemm.spgemm(tool, A, A); C.release()
    print(f"[{time.time()-t0:.1f}s] call {i}: numeric {t.Numeric:.3f} ms", flush=True)
    if hasattr(L, "mhs_diag_guard"):  # probe-guard trips (a key missing from its hash table)
        L.mhs_diag_guard(g)
        print(f"  probe guard: trips {g[0]} first: where {g[1]} key {g[2]} H {g[3]}", flush=True)
buf = np.zeros(A.M * 8, np.uint64)
assert L.mhs_memcpy(tool.ctx, ctypes.c_void_p(buf.ctypes.data), dev, buf.nbytes, 1) == 0
ph = buf.reshape(A.M, 8).astype(np.float64)
heads = ph[:, :8].sum(1) > 0
names = ["prologue", "tiles(load/build)", "bases", "clear_acc", "accumulate", "output(cols)"]
print("heads", heads.sum(), "of", A.M, flush=True)
if ph[heads, 6:8].sum() > 0:  # table rows split their output: values [6], column staging [7], columns [5]
    print(f"{'output: values':20s} {ph[heads, 6].mean():10.0f} cycles/head")
    print(f"{'output: col staging':20s} {ph[heads, 7].mean():10.0f} cycles/head")
for k, nm in enumerate(names):
    print(f"{nm:20s} {ph[heads, k].mean():10.0f} cycles/head")
tot = ph[heads, :8].sum()
print("sum cycles over heads %.3e ; numeric ms %.4f" % (tot, t.Numeric))
tot_r = ph[:, :8].sum(1)
thr = np.percentile(tot_r[heads], 99)
slow = heads & (tot_r >= thr)
print("slowest 1%% rows: %d rows, mean total %.0f cycles" % (slow.sum(), tot_r[slow].mean()))
for k, nm in enumerate(names):
    print(f"  {nm:20s} {ph[slow, k].mean():10.0f} cycles/row")
lo_, hi_ = np.percentile(tot_r[heads], [25, 75])
mid = heads & (tot_r >= lo_) & (tot_r <= hi_)
print("middle 50%% rows: %d rows, mean total %.0f cycles" % (mid.sum(), tot_r[mid].mean()))
for k, nm in enumerate(names):
    print(f"  {nm:20s} {ph[mid, k].mean():10.0f} cycles/row")
blen = np.diff(A.ptr).astype(np.int64)
rf = np.add.reduceat(blen[A.col], A.ptr[:-1]) * (np.diff(A.ptr) > 0)
edges = [0, 256, 1024, 2048, 4096, 8192, 1 << 40]
for a_, b_ in zip(edges[:-1], edges[1:]):
    sel = heads & (rf >= a_) & (rf < b_)
    if sel.sum() == 0:
        continue
    print("flop [%d, %d): %d rows, mean total %.0f cycles:" % (a_, b_, sel.sum(), tot_r[sel].mean()),
          " ".join(f"{nm.split('(')[0]}={ph[sel, k].mean():.0f}" for k, nm in enumerate(names)))
# the ten slowest rows (hub rows: is one row the launch's tail?)
Cp = None
order = np.argsort(-tot_r)[:10]
nA = np.diff(A.ptr)
print("slowest rows: row, total cycles (ms at 2.4 GHz), flop, nA, phases")
for r in order:
    print(f"  {r:9d} {tot_r[r]:12.0f} ({tot_r[r] / 2.4e6:.3f} ms) flop {rf[r]:9d} nA {nA[r]:6d} ",
          " ".join(f"{ph[r, k]:.0f}" for k in range(6)))

if sdev.value:
    sb = np.zeros(A.M * 4, np.uint64)
    assert L.mhs_memcpy(tool.ctx, ctypes.c_void_p(sb.ctypes.data), sdev, sb.nbytes, 1) == 0
    sp_ = sb.reshape(A.M, 4).astype(np.float64)
    srow = sp_.sum(1) > 0
    snames = ["clear", "tile walk", "count", "cache/spill"]
    print("symbolic table rows", srow.sum(), "of", A.M)
    for k, nm in enumerate(snames):
        print(f"  {nm:12s} {sp_[srow, k].mean():10.0f} cycles/row")
    tot_s = sp_.sum(1)
    print("slowest symbolic rows: row, total cycles, flop, nA, phases")
    for r in np.argsort(-tot_s)[:10]:
        print(f"  {r:9d} {tot_s[r]:12.0f} flop {rf[r]:9d} nA {nA[r]:6d} ", " ".join(f"{sp_[r, k]:.0f}" for k in range(4)))
