"""Host-side mirror of the reference's SpGEMM interface, over the C-ABI.

Names, argument meaning and error behaviour follow the reference
(yyssys/MH-SpGEMM):

  * ``CSR``            inc/CSR.h:4-44, src/CSR.cu -- host arrays (numpy) plus device
                       arrays, ``H2D()``, ``D2H()``, ``==`` (src/CSR.cu:48-96: raises
                       on an nnz mismatch or more than 10 errors, like the C++ throws).
  * ``Timing``         inc/Timing.h, src/Timing.cpp -- the 7 phase fields, ``getTotal()``
                       (without Form_mask_matrix_B), ``print_step_time()``.
  * ``Tool``           inc/Tool.h -- here it owns the C-ABI context (stream, workspace).
  * ``MH_spgemm``      src/main.cu:12-72 -- C = A * B on device-resident A, B.
  * ``readMtxFile``    inc/mmio_read.h:34-159.

Device memory for A and B comes from PyTorch (HIP allocations on ``cuda:N``);
C is allocated by the library.  No torch type crosses the ABI: only pointers.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass, field

import numpy as np

from . import _lib as L


class MHSpGEMMError(RuntimeError):
    """A C-ABI call returned a non-zero mhs_status (the reference throws std::exception)."""

    def __init__(self, status: int, msg: str):
        super().__init__(f"{L.STATUS_NAMES.get(status, status)}: {msg}")
        self.status = status


def _check(ctx, rc: int, what: str):
    if rc != L.MHS_OK:
        msg = L.lib().mhs_last_error(ctx).decode() if ctx else what
        raise MHSpGEMMError(rc, f"{what}: {msg}")


def _torch():
    import torch
    return torch


# ----------------------------------------------------------------- context ---

class Tool:
    """The reference's Tool (inc/Tool.h): here the C-ABI context of one device."""

    def __init__(self, device: int = 0):
        self.device = device
        self.ctx = ctypes.c_void_p()
        _check(None, L.lib().mhs_ctx_create(ctypes.byref(self.ctx), device), "mhs_ctx_create")

    def set_stream(self, hip_stream: int | None):
        _check(self.ctx, L.lib().mhs_ctx_set_stream(self.ctx, hip_stream or None), "mhs_ctx_set_stream")

    def set_option(self, option: int, value: int):
        """mhs_ctx_set_option: MHS_OPT_SYNC (0: return once the numeric phase is
        queued) or MHS_OPT_NUMERIC_EVENTS (ring size of numeric-phase events)."""
        _check(self.ctx, L.lib().mhs_ctx_set_option(self.ctx, option, value), "mhs_ctx_set_option")

    def numeric_ms(self, n: int) -> list[float]:
        """Numeric-phase durations (ms) of the last n calls (hipEvents on the stream)."""
        buf = (ctypes.c_float * max(1, n))()
        k = L.lib().mhs_ctx_numeric_ms(self.ctx, buf, n)
        if k < 0:
            _check(self.ctx, -k, "mhs_ctx_numeric_ms")
        return [float(buf[i]) for i in range(k)]

    def probe_conflicts(self) -> int:
        """Hash probe conflicts since the last query (the reference's HASH_CONFLICT count,
        src/main.cu:68-71); needs the diagnostic library (MHS_LIB=.../libmhspgemm_probe.so)."""
        v = ctypes.c_uint64()
        _check(self.ctx, L.lib().mhs_probe_conflicts(self.ctx, ctypes.byref(v)), "mhs_probe_conflicts")
        return int(v.value)

    def chunked_calls(self) -> int:
        """Calls that ran row-chunked (the out-of-memory fallback)."""
        return int(L.lib().mhs_ctx_chunked_calls(self.ctx))

    STATS = {"chunked": 0, "split": 1, "sym_fork": 2, "nft": 3, "near": 4, "multi_stream": 5,
             "spec": 6, "spec_miss": 7, "spec_skipped": 8}

    def stat(self, name: str) -> int:
        """Calls of this context that took a path (mhs_ctx_stat: 'split', 'sym_fork', 'nft',
        'near', 'multi_stream', 'chunked')."""
        return int(L.lib().mhs_ctx_stat(self.ctx, self.STATS[name]))

    def hbm_peak(self, nbytes: int = 2 << 30, iters: int = 10) -> dict:
        """Measured HBM bandwidth of this device (GB/s): copy (read + write bytes), read,
        write streaming kernels over `nbytes` buffers (mhs_hbm_peak)."""
        out = (ctypes.c_double * 3)()
        _check(self.ctx, L.lib().mhs_hbm_peak(self.ctx, nbytes, iters, out), "mhs_hbm_peak")
        return {"copy_GBps": round(out[0], 1), "read_GBps": round(out[1], 1), "write_GBps": round(out[2], 1),
                "buffer_bytes": int(nbytes), "iters": int(iters)}

    def allocate(self, B=None, C=None):  # src/Tool.cu:4 -- workspace grows on demand
        return None

    def release(self):
        if self.ctx:
            L.lib().mhs_ctx_trim(self.ctx)

    def close(self):
        if self.ctx:
            L.lib().mhs_ctx_destroy(self.ctx)
            self.ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


@dataclass
class Timing:
    """Reference Timing (inc/Timing.h:3-20), ms; plus the e2e total and run stats."""
    mem_alloc: float = 0.0
    Form_mask_matrix_B: float = 0.0
    Calculate_C_nnz: float = 0.0
    Malloc_C_col_val: float = 0.0
    Numeric: float = 0.0
    symbolic_binning: float = 0.0
    numeric_binning: float = 0.0
    total_e2e: float = 0.0
    flop: int = 0
    nnzC: int = 0
    sym_bins: list = field(default_factory=lambda: [0] * 16)
    num_bins: list = field(default_factory=lambda: [0] * 16)

    PHASES = ("mem_alloc", "Form_mask_matrix_B", "Calculate_C_nnz", "Malloc_C_col_val",
              "Numeric", "symbolic_binning", "numeric_binning", "total_e2e")

    def getTotal(self) -> float:  # src/Timing.cpp:39-41: Form_mask_matrix_B excluded
        return (self.Calculate_C_nnz + self.Malloc_C_col_val + self.Numeric + self.symbolic_binning
                + self.numeric_binning + self.mem_alloc)

    def __iadd__(self, t: "Timing"):
        for k in self.PHASES:
            setattr(self, k, getattr(self, k) + getattr(t, k))
        return self

    def __itruediv__(self, x: float):
        for k in self.PHASES:
            setattr(self, k, getattr(self, k) / x)
        return self

    def print_step_time(self):
        print("  -------------time-------------")
        print(f"    mem_alloc: \t\t{self.mem_alloc:.3f}ms")
        print(f"    form_mask_matrix_B: {self.Form_mask_matrix_B:.3f}ms")
        print(f"    symbolic_binning: \t{self.symbolic_binning:.3f}ms")
        print(f"    calculate_C_nnz: \t{self.Calculate_C_nnz:.3f}ms")
        print(f"    malloc_C_col_val: \t{self.Malloc_C_col_val:.3f}ms")
        print(f"    numeric_binning: \t{self.numeric_binning:.3f}ms")
        print(f"    numeric: \t\t{self.Numeric:.3f}ms")
        print("  ------------------------------")

    @classmethod
    def from_c(cls, t: L.mhs_timing) -> "Timing":
        return cls(mem_alloc=t.mem_alloc, Form_mask_matrix_B=t.Form_mask_matrix_B,
                   Calculate_C_nnz=t.Calculate_C_nnz, Malloc_C_col_val=t.Malloc_C_col_val,
                   Numeric=t.Numeric, symbolic_binning=t.symbolic_binning,
                   numeric_binning=t.numeric_binning, total_e2e=t.total_e2e, flop=int(t.flop),
                   nnzC=int(t.nnzC), sym_bins=list(t.sym_bins), num_bins=list(t.num_bins))


# --------------------------------------------------------------------- CSR ---

class DeviceCSR:
    """A device CSR produced by the library (hipMalloc'ed); recycled into the
    context's output pool when released (the reference frees with cudaFree)."""

    def __init__(self, tool: Tool, c: L.mhs_csr):
        self.tool = tool
        self.c = c

    @property
    def M(self):
        return self.c.M

    @property
    def N(self):
        return self.c.N

    @property
    def nnz(self):
        return self.c.nnz

    def to_host(self):
        M, nnz = self.c.M, self.c.nnz
        ptr = np.empty(M + 1, np.int32)
        col = np.empty(nnz, np.int32)
        val = np.empty(nnz, np.float64)
        lib, ctx = L.lib(), self.tool.ctx
        _check(ctx, lib.mhs_memcpy(ctx, ptr.ctypes.data, self.c.ptr, ptr.nbytes, 1), "D2H ptr")
        if nnz:
            _check(ctx, lib.mhs_memcpy(ctx, col.ctypes.data, self.c.col, col.nbytes, 1), "D2H col")
            _check(ctx, lib.mhs_memcpy(ctx, val.ctypes.data, self.c.val, val.nbytes, 1), "D2H val")
        return ptr, col, val

    def to_torch(self, device=None):
        """Copy into torch tensors on the context's device (D2D)."""
        torch = _torch()
        dev = device or f"cuda:{self.tool.device}"
        ptr = torch.empty(self.c.M + 1, dtype=torch.int32, device=dev)
        col = torch.empty(self.c.nnz, dtype=torch.int32, device=dev)
        val = torch.empty(self.c.nnz, dtype=torch.float64, device=dev)
        torch.cuda.synchronize(dev)
        lib, ctx = L.lib(), self.tool.ctx
        _check(ctx, lib.mhs_memcpy(ctx, ptr.data_ptr(), self.c.ptr, 4 * (self.c.M + 1), 2), "D2D ptr")
        if self.c.nnz:
            _check(ctx, lib.mhs_memcpy(ctx, col.data_ptr(), self.c.col, 4 * self.c.nnz, 2), "D2D col")
            _check(ctx, lib.mhs_memcpy(ctx, val.data_ptr(), self.c.val, 8 * self.c.nnz, 2), "D2D val")
        return ptr, col, val

    def release(self):
        if self.c.ptr or self.c.col or self.c.val:
            if self.tool.ctx:
                L.lib().mhs_ctx_recycle(self.tool.ctx, ctypes.byref(self.c))
            else:
                L.lib().mhs_csr_free(ctypes.byref(self.c))

    def __del__(self):
        try:
            self.release()
        except Exception:
            pass


class CSR:
    """Reference CSR (inc/CSR.h): host arrays ptr/col/val (numpy), device arrays
    d_ptr/d_col/d_val (torch tensors, or a DeviceCSR for library outputs)."""

    def __init__(self, M=0, N=0, ptr=None, col=None, val=None, isSymmetric=0):
        self.M, self.N = int(M), int(N)
        self.ptr = None if ptr is None else np.ascontiguousarray(ptr, dtype=np.int32)
        self.col = None if col is None else np.ascontiguousarray(col, dtype=np.int32)
        self.val = None if val is None else np.ascontiguousarray(val, dtype=np.float64)
        self.nnz = 0 if self.col is None else int(self.col.shape[0])
        self.isSymmetric = int(isSymmetric)
        self.d_ptr = self.d_col = self.d_val = None
        self.dev: DeviceCSR | None = None

    # --- reference methods -------------------------------------------------
    def alloc(self, r, c, n):
        self.M, self.N, self.nnz = r, c, n
        self.ptr = np.zeros(r + 1, np.int32)
        self.col = np.zeros(n, np.int32)
        self.val = np.zeros(n, np.float64)

    def copy(self) -> "CSR":  # operator= (deep host copy, src/CSR.cu:34-47)
        return CSR(self.M, self.N, self.ptr.copy(), self.col.copy(), self.val.copy(), self.isSymmetric)

    def H2D(self, device: int = 0):
        torch = _torch()
        dev = f"cuda:{device}"
        self.d_ptr = torch.from_numpy(self.ptr).to(dev)
        self.d_col = torch.from_numpy(self.col).to(dev)
        self.d_val = torch.from_numpy(self.val).to(dev)
        torch.cuda.synchronize(dev)

    def D2H(self):
        if self.dev is not None:
            self.ptr, self.col, self.val = self.dev.to_host()
        else:
            self.ptr = self.d_ptr.cpu().numpy()
            self.col = self.d_col.cpu().numpy()
            self.val = self.d_val.cpu().numpy()
        self.nnz = int(self.col.shape[0])

    def d_release_csr(self):
        if self.dev is not None:
            self.dev.release()
            self.dev = None
        self.d_ptr = self.d_col = self.d_val = None

    def release(self):
        self.d_release_csr()
        self.ptr = self.col = self.val = None

    def c_view(self) -> L.mhs_csr:
        """mhs_csr over the device arrays (for the C-ABI)."""
        if self.dev is not None:
            return self.dev.c
        def p(t):
            return None if t is None or t.numel() == 0 else t.data_ptr()
        return L.mhs_csr(self.M, self.N, self.nnz, p(self.d_ptr), p(self.d_col), p(self.d_val))

    def __eq__(self, other: "CSR") -> bool:
        """CSR::operator== (src/CSR.cu:48-96), vectorised.  Raises RuntimeError
        where the reference throws (nnz mismatch, > 10 errors, ptr[M] mismatch)."""
        if self.nnz != other.nnz:
            print(f"nnz not equal {self.nnz} {other.nnz}")
            raise RuntimeError("nnz not equal")
        assert self.M == other.M and self.N == other.N, "dimension not same"
        return compare_ref(self.ptr, self.col, self.val, other.ptr, other.col, other.val)

    __hash__ = None


def compare_ref(p, c, v, p2, c2, v2, verbose=True) -> bool:
    """The reference comparison rule: ptr and col exact; val accepted when
    |d| < 1e-9 or |d| < 1e-9*|v| (v is the left operand)."""
    M = len(p) - 1
    eps = 1e-9
    if p[M] != p2[M]:
        raise RuntimeError("matrix compare: error num exceed threshold")
    bad_ptr = np.nonzero(p[:M] != p2[:M])[0]
    errs = len(bad_ptr)
    if errs == 0:
        bad_col = np.nonzero(c != c2)[0]
        d = np.abs(v - v2)
        bad_val = np.nonzero(~((d < eps) | (d < eps * np.abs(v))))[0]
        errs += len(bad_col) + len(bad_val)
        if verbose:
            for j in bad_col[:11]:
                print(f"col not equal at index {j}, {c[j]} != {c2[j]}")
            for j in bad_val[:11]:
                print(f"val not eqaul at index {j}, value {v[j]:.18e} != {v2[j]:.18e}")
    elif verbose:
        for i in bad_ptr[:11]:
            print(f"ptr not equal at {i} rows, {p[i]} != {p2[i]}")
    if errs > 10:
        raise RuntimeError("matrix compare: error num exceed threshold")
    return errs == 0


def compare_tol(p_ref, c_ref, v_ref, p, c, v, rtol=1e-6, atol=1e-12):
    """North-star parity: ptr and col bit-exact, |dv| <= rtol*|ref| or <= atol.
    Returns (ok, n_bad_ptr, n_bad_col, n_bad_val, max_rel)."""
    if len(p_ref) != len(p) or p_ref[-1] != p[-1]:
        return False, -1, -1, -1, float("inf")
    bp = int(np.count_nonzero(p_ref != p))
    bc = int(np.count_nonzero(c_ref != c))
    d = np.abs(v_ref - v)
    ok_v = (d <= atol) | (d <= rtol * np.abs(v_ref))
    bv = int(np.count_nonzero(~ok_v))
    with np.errstate(divide="ignore", invalid="ignore"):
        rel = np.where(np.abs(v_ref) > 0, d / np.abs(v_ref), d)
    mr = float(rel.max()) if rel.size else 0.0
    return (bp == 0 and bc == 0 and bv == 0), bp, bc, bv, mr


# ------------------------------------------------------------- entry points ---

def spgemm(tool: Tool, A: CSR, B: CSR, timing: bool = True):
    """C = A * B with A, B device-resident (H2D done).  Returns (DeviceCSR, Timing|None)."""
    a, b = A.c_view(), B.c_view()
    c = L.mhs_csr()
    t = L.mhs_timing() if timing else None
    rc = L.lib().mhs_spgemm(tool.ctx, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c),
                            ctypes.byref(t) if t is not None else None)
    _check(tool.ctx, rc, "mhs_spgemm")
    return DeviceCSR(tool, c), (Timing.from_c(t) if t is not None else None)


def transpose(tool: Tool, A: CSR) -> CSR:
    """A^T on the device (mhs_transpose): the AAT operand B = transpose(A)
    (src/main.cu:98-99, host version src/utils.cpp:20-46).  A must be device-
    resident; the result's device arrays are a library-owned DeviceCSR."""
    a = A.c_view()
    t = L.mhs_csr()
    _check(tool.ctx, L.lib().mhs_transpose(tool.ctx, ctypes.byref(a), ctypes.byref(t)), "mhs_transpose")
    out = CSR(t.M, t.N)
    out.nnz = t.nnz
    out.dev = DeviceCSR(tool, t)
    return out


def matrix_transposition(A: CSR, B: CSR, tool: Tool | None = None) -> None:
    """src/utils.cpp:20-46 (B = A^T, host arrays) computed on the device: A is
    uploaded if needed, transposed with mhs_transpose, and B gets host arrays."""
    own = tool is None
    tool = tool or Tool(0)
    try:
        if A.dev is None and A.d_ptr is None:
            A.H2D(tool.device)
        T = transpose(tool, A)
        B.M, B.N, B.nnz = T.M, T.N, T.nnz
        B.ptr, B.col, B.val = T.dev.to_host()
        B.isSymmetric = 0
        T.d_release_csr()
    finally:
        if own:
            tool.close()


def vendor_spgemm(tool: Tool, A: CSR, B: CSR, warmup: int = 0):
    """rocSPARSE C = A * B (include/mhs_vendor.h; the reference's cusparse_spgemm,
    inc/cusparse_spgemm.cuh:94-105).  `warmup` untimed calls first (rocSPARSE loads its
    code objects on first use).  Returns (DeviceCSR, ms over the reference's span)."""
    V = L.vendor_lib()
    a, b = A.c_view(), B.c_view()
    for i in range(warmup + 1):
        c = L.mhs_csr()
        ms = ctypes.c_double(0.0)
        err = ctypes.create_string_buffer(256)
        rc = V.mhs_vendor_spgemm(tool.device, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c),
                                 ctypes.byref(ms), err, 256)
        if rc != L.MHS_OK:
            raise MHSpGEMMError(rc, f"rocSPARSE SpGEMM: {err.value.decode(errors='replace')}")
        if i < warmup:
            V.mhs_vendor_free(ctypes.byref(c))
    return DeviceCSR(tool, c), float(ms.value)


def MH_spgemm(A: CSR, B: CSR, C: CSR, timing: Timing, tools: Tool):
    """src/main.cu:12-72: C.M = A.M, C.N = B.N, C.nnz and C's device arrays set;
    phase times written into `timing`.  Raises MHSpGEMMError on failure."""
    if tools.device is not None:
        try:
            torch = _torch()
            tools.set_stream(torch.cuda.current_stream(tools.device).cuda_stream)
        except Exception:
            tools.set_stream(None)
    dev, t = spgemm(tools, A, B, timing=True)
    C.d_release_csr()
    C.dev = dev
    C.M, C.N, C.nnz = dev.M, dev.N, dev.nnz
    for k in Timing.PHASES + ("flop", "nnzC", "sym_bins", "num_bins"):
        setattr(timing, k, getattr(t, k))
    print(f"C.nnz = {C.nnz}")


def _cache_setting(v):
    """$MHS_MTX_CACHE: unset, "", "0", "false", "no", "off" -> off; "1", "true", "yes", "on" ->
    next to the file; anything else -> a cache directory."""
    if v is None or v.strip().lower() in ("", "0", "false", "no", "off"):
        return False
    if v.strip().lower() in ("1", "true", "yes", "on"):
        return True
    return v


def readMtxFile(A: CSR, filename: str, cache=None) -> int:
    """inc/mmio_read.h:34-159 through the library's parallel reader.

    ``cache`` (default ``$MHS_MTX_CACHE``: unset = off, "1" = next to the file,
    else a directory): read a binary CSR cache stamped with the .mtx's size and
    mtime instead of the text, writing it on a miss."""
    h = L.mhs_host_csr()
    if cache is None:
        cache = _cache_setting(os.environ.get("MHS_MTX_CACHE"))
    if cache and cache is not True and str(cache).lower() not in ("1", "true", "yes", "on"):
        d = os.fspath(cache)
        os.makedirs(d, exist_ok=True)
        cpath = os.path.join(d, os.path.basename(str(filename)) + ".mhscsr").encode()
    else:
        cpath = None
    if cache:
        hit = ctypes.c_int(0)
        rc = L.lib().mhs_read_mtx_cached(str(filename).encode(), cpath, ctypes.byref(h), ctypes.byref(hit))
        readMtxFile.last_from_cache = bool(hit.value)
    else:
        rc = L.lib().mhs_read_mtx(str(filename).encode(), ctypes.byref(h))
        readMtxFile.last_from_cache = False
    if rc != L.MHS_OK:
        print(f"Could not read Matrix Market file {filename}.")
        return -1
    try:
        M, nnz = h.M, h.nnz
        ptr = np.ctypeslib.as_array(ctypes.cast(h.ptr, ctypes.POINTER(ctypes.c_int32)), (M + 1,)).copy()
        if nnz:
            col = np.ctypeslib.as_array(ctypes.cast(h.col, ctypes.POINTER(ctypes.c_int32)), (nnz,)).copy()
            val = np.ctypeslib.as_array(ctypes.cast(h.val, ctypes.POINTER(ctypes.c_double)), (nnz,)).copy()
        else:
            col = np.zeros(0, np.int32)
            val = np.zeros(0, np.float64)
        A.M, A.N, A.nnz = h.M, h.N, nnz
        A.ptr, A.col, A.val = ptr, col, val
        A.isSymmetric = h.is_symmetric
    finally:
        L.lib().mhs_host_csr_free(ctypes.byref(h))
    return 0


def flop_count(A: CSR, B: CSR) -> int:
    """int_result of src/main.cu:102-107 (sum of B row lengths over A's nonzeros)."""
    return int(L.lib().mhs_flop_count(A.nnz, A.col.ctypes.data, B.ptr.ctypes.data))


def flop_count_np(Acol: np.ndarray, Bptr: np.ndarray) -> int:
    blen = np.diff(Bptr.astype(np.int64))
    return int(blen[Acol].sum()) if len(Acol) else 0
