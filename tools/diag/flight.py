"""Flight recorder run of the stamps build (tools/diag/build.sh: -DMHS_ROW_STAMPS=1): every wave of
the numeric wave kernels writes its current row, list index, last phase stamp and a tick to
fine-grained host memory; the product call runs in a thread, and if it has not returned after
--wait seconds this prints the waves that are inside a row (phase < 6) with the rows' shapes, then
ends the process (the driver tears the queue down).  usage:
  STAMPS_LIB=tools/diag/v9/libmhspgemm.so python tools/diag/flight.py cage15-r5 [--wait 40] [--calls 3]"""
import argparse, ctypes, os, sys, threading, time
from pathlib import Path
ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "mh-spgemm_amd")]
os.environ["MHS_LIB"] = os.environ.get("STAMPS_LIB", str(ROOT / "tools/diag/v9/libmhspgemm.so"))
ap = argparse.ArgumentParser()
ap.add_argument("matrix")
ap.add_argument("--wait", type=float, default=40.0)
ap.add_argument("--calls", type=int, default=3)
args = ap.parse_args()
import numpy as np, torch  # noqa: E402
import mhspgemm  # noqa: E402
from mhspgemm import _lib, synth  # noqa: E402
t0 = time.time()
A, _ = synth.load_or_synth(args.matrix)
print(f"[{time.time()-t0:.1f}s] matrix {args.matrix} rows {A.M}", flush=True)
A.H2D(0)
tool = mhspgemm.Tool(0)
L = _lib.lib()
L.mhs_diag_setup.argtypes = [ctypes.c_int, ctypes.c_void_p]
dev = ctypes.c_void_p()
assert L.mhs_diag_setup(A.M, ctypes.byref(dev)) == 0
hip = ctypes.CDLL("libamdhip64.so.7" if os.path.exists("/opt/rocm/lib/libamdhip64.so.7") else "libamdhip64.so")
NW = 65536
host = ctypes.c_void_p()
assert hip.hipHostMalloc(ctypes.byref(host), ctypes.c_size_t(NW * 32), ctypes.c_uint(0x2 | 0x40000000)) == 0
ctypes.memset(host, 0, NW * 32)
dptr = ctypes.c_void_p()
assert hip.hipHostGetDevicePointer(ctypes.byref(dptr), host, ctypes.c_uint(0)) == 0
L.mhs_diag_flight.argtypes = [ctypes.c_void_p]
assert L.mhs_diag_flight(dptr) == 0
fl = np.ctypeslib.as_array(ctypes.cast(host, ctypes.POINTER(ctypes.c_uint64)), shape=(NW, 4))
rows_h = None
if os.environ.get("FLIGHT_HOST_ROWS"):  # the row stamps themselves in host memory (no extra code)
    rh = ctypes.c_void_p()
    assert hip.hipHostMalloc(ctypes.byref(rh), ctypes.c_size_t(A.M * 64), ctypes.c_uint(0x2 | 0x40000000)) == 0
    ctypes.memset(rh, 0, A.M * 64)
    rd = ctypes.c_void_p()
    assert hip.hipHostGetDevicePointer(ctypes.byref(rd), rh, ctypes.c_uint(0)) == 0
    L.mhs_diag_set_rows.argtypes = [ctypes.c_void_p]
    assert L.mhs_diag_set_rows(rd) == 0
    rows_h = np.ctypeslib.as_array(ctypes.cast(rh, ctypes.POINTER(ctypes.c_uint64)), shape=(A.M, 8))
done = []


def work():
    for i in range(args.calls):
        C, t = mhspgemm.spgemm(tool, A, A)
        C.release()
        done.append(t.Numeric)
        print(f"[{time.time()-t0:.1f}s] call {i}: numeric {t.Numeric:.3f} ms", flush=True)


th = threading.Thread(target=work, daemon=True)
th.start()
th.join(args.wait)
if not th.is_alive():
    print("FLIGHT: every call returned", flush=True)
    sys.exit(0)
snap = fl.copy()
time.sleep(2.0)
snap2 = fl.copy()
live = (snap[:, 2] != 0)
inrow = live & (snap[:, 1] < 6)
moving = (snap2[:, 2] != snap[:, 2]) | (snap2[:, 3] != snap[:, 3])
print(f"FLIGHT: call {len(done)} still running after {args.wait:.0f} s; waves recorded {live.sum()}, "
      f"inside a row {inrow.sum()}, still moving {moving.sum()}", flush=True)
nA = np.diff(A.ptr)
blen = nA.astype(np.int64)
for w in np.nonzero(inrow)[0][:40]:
    row = int(snap[w, 0] & 0xFFFFFFFF)
    li = int(snap[w, 0] >> 32)
    cols = A.col[A.ptr[row]:A.ptr[row + 1]] if row < A.M else np.zeros(0, np.int32)
    flop = int(blen[cols].sum()) if len(cols) else -1
    span = (int(cols.max() >> 6) - int(cols.min() >> 6) + 1) if len(cols) else -1
    print(f"  wave {w}: row {row} li {li} phase {int(snap[w, 1]) - 1} last take {int(snap[w, 3])} "
          f"tick {int(snap[w, 2])} moving {bool(moving[w])} | nA {int(nA[row]) if row < A.M else -1} flop {flop} "
          f"A-span tiles {span}", flush=True)
if rows_h is not None:
    st = rows_h[:, :6].copy()
    started = (st != 0).any(1)
    part = started & ~(st != 0).all(1)
    print(f"ROWS: started {started.sum()} of {A.M}, partial {part.sum()}", flush=True)
    for r in np.nonzero(part)[0][:40]:
        cols = A.col[A.ptr[r]:A.ptr[r + 1]]
        flop = int(blen[cols].sum()) if len(cols) else 0
        span = (int(cols.max() >> 6) - int(cols.min() >> 6) + 1) if len(cols) else 0
        print(f"  row {r}: stamps {[int(x) for x in st[r]]} nA {int(nA[r])} flop {flop} A-span tiles {span}", flush=True)
print("FLIGHT: exiting with the kernel still running", flush=True)
os._exit(3)
