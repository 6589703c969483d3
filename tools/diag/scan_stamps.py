"""Phase stamps of k_scan and k_bin_list per block (diagnostic build -DMHS_SCAN_STAMPS=1):
  python tools/diag/scan_stamps.py <matrix>   (SCAN_LIB=<dir>/libmhspgemm.so)
Prints, over the blocks of the last call, the median cycles of each phase and when the blocks
start / finish relative to the first block's start."""
import ctypes, os, sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "mh-spgemm_amd")]
os.environ["MHS_LIB"] = os.environ.get("SCAN_LIB", str(ROOT / "ablib/scanstamps/libmhspgemm.so"))
import numpy as np, torch  # noqa: E402
import mhspgemm  # noqa: E402
from mhspgemm import _lib, synth  # noqa: E402
name = sys.argv[1]
A, _ = synth.load_or_synth(name)
A.H2D(0)
tool = mhspgemm.Tool(0)
L = _lib.lib()
L.mhs_diag_setup_scan.argtypes = [ctypes.c_int, ctypes.c_void_p]
nb = (A.M + 1 + 1023) // 1024 + 8
dev = ctypes.c_void_p()
assert L.mhs_diag_setup_scan(nb, ctypes.byref(dev)) == 0
for _ in range(4):
    C, t = mhspgemm.spgemm(tool, A, A)
    C.release()
buf = np.zeros(nb * 16, np.uint64)
assert L.mhs_memcpy(tool.ctx, ctypes.c_void_p(buf.ctypes.data), dev, buf.nbytes, 1) == 0
st = buf.reshape(nb, 16).astype(np.int64)
for lo, hi, names in ((0, 8, ["start", "counts+scan", "classify", "look-back", "row_ptr", "append", "last", "publish"]),
                      (8, 11, ["start", "classify", "append"])):
    s = st[:, lo:hi]
    live = s[:, 0] > 0
    s = s[live]
    t0 = s[:, 0].min()
    print(f"{'k_scan' if lo == 0 else 'k_bin_list'}: {live.sum()} blocks; block start spread {np.median(s[:, 0] - t0):.0f} "
          f"(median) / {(s[:, 0] - t0).max()} (max) cycles after the first")
    for k in range(1, hi - lo):
        d = s[:, k] - s[:, k - 1]
        ok = (s[:, k] > 0) & (s[:, k - 1] > 0)
        if ok.any():
            print(f"   {names[k - 1]:>12s} -> {names[k]:<12s} median {np.median(d[ok]):9.0f}  max {d[ok].max():9.0f} cycles")
    ends = s[:, hi - lo - 1]
    ends = ends[ends > 0]
    print(f"   last stamp of the last block: {ends.max() - t0} cycles after the first start; phases: {t.numeric_binning:.4f} ms numeric_binning")
