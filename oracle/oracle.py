"""ctypes wrapper of oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module, and only as the checker / the CPU baseline.  It restates the
reference host semantics (see oracle.h for the file:line of each function):
  read_mtx    inc/mmio_read.h:34-159, inc/mmio.h:128-232
  flop        src/main.cu:102-107
  transpose   src/utils.cpp:20-46
  spgemm      Gustavson, structural nnz, sorted columns, fixed-order FP64 sums
              (the result contract of inc/Calculate_C_nnz.cuh + inc/numeric.cuh)
  compare_ref CSR::operator== (src/CSR.cu:48-96)

Parity status: UNPINNED against reference-generated outputs (the reference has
no tests or fixtures for this path and cannot be built here -- DESIGN.md
§Oracle); pinned bit-exactly to scipy.sparse fixtures (tests/golden/) and to
hand-derived known answers.
"""
from __future__ import annotations

import ctypes
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
SO = HERE / "liboracle.so"

_lib = None


class orc_csr(ctypes.Structure):
    _fields_ = [("M", ctypes.c_int32), ("N", ctypes.c_int32), ("nnz", ctypes.c_int32),
                ("ptr", ctypes.c_void_p), ("col", ctypes.c_void_p), ("val", ctypes.c_void_p),
                ("is_symmetric", ctypes.c_int32)]


def build():
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)


def lib():
    global _lib
    if _lib is None:
        if not SO.exists():
            build()
        L = ctypes.CDLL(str(SO))
        vp, i32, i64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
        L.orc_read_mtx.argtypes = [ctypes.c_char_p, ctypes.POINTER(orc_csr)]
        L.orc_read_mtx.restype = ctypes.c_int
        L.orc_csr_free.argtypes = [ctypes.POINTER(orc_csr)]
        L.orc_flop.argtypes = [i32, vp, vp]
        L.orc_flop.restype = ctypes.c_ulonglong
        L.orc_transpose.argtypes = [ctypes.POINTER(orc_csr), ctypes.POINTER(orc_csr)]
        L.orc_spgemm_symbolic.argtypes = [i32, i32, vp, vp, vp, vp, vp, ctypes.c_int]
        L.orc_spgemm_symbolic.restype = i64
        L.orc_spgemm_numeric.argtypes = [i32, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp, i32, i32,
                                         ctypes.c_int]
        L.orc_spgemm_numeric.restype = ctypes.c_int
        L.orc_compare_ref.argtypes = [i32, i32, vp, vp, vp, i32, vp, vp, vp, ctypes.c_int]
        L.orc_compare_ref.restype = ctypes.c_int
        L.orc_compare_tol.argtypes = [i32, i32, vp, vp, vp, i32, vp, vp, vp, ctypes.c_double,
                                      ctypes.c_double]
        L.orc_compare_tol.restype = i64
        L.orc_max_threads.restype = ctypes.c_int
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data if a is not None and a.size else None


def _arr(ptr, n, dt):
    if n == 0:
        return np.zeros(0, dt)
    ct = ctypes.c_int32 if dt == np.int32 else ctypes.c_double
    return np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(ct)), (n,)).copy()


def read_mtx(path: str):
    """-> (M, N, ptr, col, val, is_symmetric) or raises OSError(code)."""
    L = lib()
    A = orc_csr()
    rc = L.orc_read_mtx(str(path).encode(), ctypes.byref(A))
    if rc != 0:
        raise OSError(rc, f"orc_read_mtx failed ({rc}) for {path}")
    try:
        return (A.M, A.N, _arr(A.ptr, A.M + 1, np.int32), _arr(A.col, A.nnz, np.int32),
                _arr(A.val, A.nnz, np.float64), A.is_symmetric)
    finally:
        L.orc_csr_free(ctypes.byref(A))


def flop(Acol, Bptr) -> int:
    Acol = np.ascontiguousarray(Acol, np.int32)
    Bptr = np.ascontiguousarray(Bptr, np.int32)
    return int(lib().orc_flop(len(Acol), _p(Acol), _p(Bptr)))


def transpose(M, N, ptr, col, val):
    L = lib()
    A = orc_csr(M, N, len(col), _p(ptr), _p(col), _p(val), 0)
    T = orc_csr()
    if L.orc_transpose(ctypes.byref(A), ctypes.byref(T)) != 0:
        raise MemoryError("orc_transpose")
    try:
        return (T.M, T.N, _arr(T.ptr, T.M + 1, np.int32), _arr(T.col, T.nnz, np.int32),
                _arr(T.val, T.nnz, np.float64))
    finally:
        L.orc_csr_free(ctypes.byref(T))


def spgemm(Ap, Ai, Av, Bp, Bi, Bv, N, nthreads=0, rows=None):
    """C = A*B.  Returns (Cp, Ci, Cv).  rows=(r0, r1) computes values only for
    that row range (Cp is always complete)."""
    L = lib()
    Ap, Ai, Av = (np.ascontiguousarray(x) for x in (Ap, Ai, Av))
    Bp, Bi, Bv = (np.ascontiguousarray(x) for x in (Bp, Bi, Bv))
    M = len(Ap) - 1
    Cp = np.empty(M + 1, np.int32)
    nnz = L.orc_spgemm_symbolic(M, N, _p(Ap), _p(Ai), _p(Bp), _p(Bi), _p(Cp), nthreads)
    if nnz < 0:
        raise MemoryError("orc_spgemm_symbolic")
    Ci = np.empty(nnz, np.int32)
    Cv = np.empty(nnz, np.float64)
    r0, r1 = (0, M) if rows is None else rows
    rc = L.orc_spgemm_numeric(M, N, _p(Ap), _p(Ai), _p(Av), _p(Bp), _p(Bi), _p(Bv), _p(Cp),
                              _p(Ci), _p(Cv), r0, r1, nthreads)
    if rc != 0:
        raise MemoryError("orc_spgemm_numeric")
    return Cp, Ci, Cv


def spgemm_symbolic(Ap, Ai, Bp, Bi, N, nthreads=0):
    L = lib()
    M = len(Ap) - 1
    Cp = np.empty(M + 1, np.int32)
    nnz = L.orc_spgemm_symbolic(M, N, _p(Ap), _p(Ai), _p(Bp), _p(Bi), _p(Cp), nthreads)
    if nnz < 0:
        raise MemoryError("orc_spgemm_symbolic")
    return Cp


def spgemm_numeric_rows(Ap, Ai, Av, Bp, Bi, Bv, N, Cp, Ci, Cv, r0, r1, nthreads=0):
    M = len(Ap) - 1
    rc = lib().orc_spgemm_numeric(M, N, _p(Ap), _p(Ai), _p(Av), _p(Bp), _p(Bi), _p(Bv), _p(Cp),
                                  _p(Ci), _p(Cv), r0, r1, nthreads)
    if rc != 0:
        raise MemoryError("orc_spgemm_numeric")


def compare_ref(p1, c1, v1, p2, c2, v2, verbose=False) -> int:
    M = len(p1) - 1
    return lib().orc_compare_ref(M, len(c1), _p(p1), _p(c1), _p(v1), len(c2), _p(p2), _p(c2),
                                 _p(v2), int(verbose))


def compare_tol(p_ref, c_ref, v_ref, p, c, v, rtol=1e-6, atol=1e-12) -> int:
    M = len(p_ref) - 1
    return int(lib().orc_compare_tol(M, len(c_ref), _p(p_ref), _p(c_ref), _p(v_ref), len(c),
                                     _p(p), _p(c), _p(v), rtol, atol))


def max_threads() -> int:
    return int(lib().orc_max_threads())
