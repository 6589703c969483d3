"""ctypes binding of libmhspgemm.so (the C-ABI declared in include/mhspgemm.h).

The shared library is built in-tree (``make -C mh-spgemm_amd``) and loaded from
this directory.  There is no fallback: if the library is missing, importing the
package raises, so no caller can silently run anything but the HIP path.
"""
from __future__ import annotations

import ctypes
import os
import re
from pathlib import Path

HERE = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ["MHS_LIB"]) if os.environ.get("MHS_LIB") else HERE / "libmhspgemm.so"
HEADER = HERE.parent.parent / "include" / "mhspgemm.h"

MHS_OK = 0
MHS_ERR_HIP = 1
MHS_ERR_OOM = 2
MHS_ERR_INVALID = 3
MHS_ERR_OVERFLOW = 4
MHS_ERR_IO = 5

MHS_OPT_SYNC = 1
MHS_OPT_NUMERIC_EVENTS = 2
MHS_OPT_MEM_BUDGET = 3
MHS_OPT_TINY_FIRST_ROWS = 4
MHS_OPT_SPECULATE = 5

STATUS_NAMES = {0: "MHS_OK", 1: "MHS_ERR_HIP", 2: "MHS_ERR_OOM", 3: "MHS_ERR_INVALID",
                4: "MHS_ERR_OVERFLOW", 5: "MHS_ERR_IO"}


class mhs_csr(ctypes.Structure):
    _fields_ = [("M", ctypes.c_int32), ("N", ctypes.c_int32), ("nnz", ctypes.c_int32),
                ("ptr", ctypes.c_void_p), ("col", ctypes.c_void_p), ("val", ctypes.c_void_p)]


class mhs_timing(ctypes.Structure):
    _fields_ = [("mem_alloc", ctypes.c_double), ("Form_mask_matrix_B", ctypes.c_double),
                ("symbolic_binning", ctypes.c_double), ("Calculate_C_nnz", ctypes.c_double),
                ("numeric_binning", ctypes.c_double), ("Malloc_C_col_val", ctypes.c_double),
                ("Numeric", ctypes.c_double), ("total_ref", ctypes.c_double),
                ("total_e2e", ctypes.c_double), ("flop", ctypes.c_uint64), ("nnzC", ctypes.c_int64),
                ("sym_bins", ctypes.c_int32 * 16), ("num_bins", ctypes.c_int32 * 16)]


class mhs_host_csr(ctypes.Structure):
    _fields_ = [("M", ctypes.c_int32), ("N", ctypes.c_int32), ("nnz", ctypes.c_int32),
                ("ptr", ctypes.c_void_p), ("col", ctypes.c_void_p), ("val", ctypes.c_void_p),
                ("is_symmetric", ctypes.c_int32)]


def declared_functions(header: Path | None = None) -> list[str]:
    """Names of the functions include/mhspgemm.h (or `header`) declares."""
    text = (header or HEADER).read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(mhs_[a-z0-9_]+)\s*\(", text)))


_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise ImportError(
            f"{LIB_PATH} is missing: build the HIP extension first "
            "(python -c 'import __graft_entry__ as g; g.build()' or make -C mh-spgemm_amd)")
    # One HIP runtime per process: PyTorch-ROCm bundles its own libamdhip64 /
    # libhsa-runtime64 (same SONAMEs as /opt/rocm's).  Loading torch first makes
    # the dynamic loader bind our NEEDED libamdhip64.so.7 to the copy already in
    # the process; the other order maps two HSA runtimes and the second one
    # finds no device.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(str(LIB_PATH))
    c_int, c_void_p, c_size_t = ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t
    P = ctypes.POINTER
    L.mhs_abi_version.restype = c_int
    L.mhs_ctx_create.argtypes = [P(c_void_p), c_int]
    L.mhs_ctx_create.restype = c_int
    L.mhs_ctx_destroy.argtypes = [c_void_p]
    L.mhs_ctx_destroy.restype = None
    L.mhs_last_error.argtypes = [c_void_p]
    L.mhs_last_error.restype = ctypes.c_char_p
    L.mhs_ctx_set_stream.argtypes = [c_void_p, c_void_p]
    L.mhs_ctx_set_stream.restype = c_int
    L.mhs_ctx_trim.argtypes = [c_void_p]
    L.mhs_ctx_trim.restype = c_int
    L.mhs_spgemm.argtypes = [c_void_p, P(mhs_csr), P(mhs_csr), P(mhs_csr), P(mhs_timing)]
    L.mhs_spgemm.restype = c_int
    L.mhs_csr_free.argtypes = [P(mhs_csr)]
    L.mhs_csr_free.restype = None
    L.mhs_ctx_recycle.argtypes = [c_void_p, P(mhs_csr)]
    L.mhs_ctx_recycle.restype = None
    L.mhs_read_mtx.argtypes = [ctypes.c_char_p, P(mhs_host_csr)]
    L.mhs_read_mtx.restype = c_int
    L.mhs_host_csr_free.argtypes = [P(mhs_host_csr)]
    L.mhs_host_csr_free.restype = None
    L.mhs_read_mtx_cached.argtypes = [ctypes.c_char_p, ctypes.c_char_p, P(mhs_host_csr), P(c_int)]
    L.mhs_read_mtx_cached.restype = c_int
    L.mhs_write_csr_bin.argtypes = [ctypes.c_char_p, P(mhs_host_csr), ctypes.c_int64, ctypes.c_int64]
    L.mhs_write_csr_bin.restype = c_int
    L.mhs_read_csr_bin.argtypes = [ctypes.c_char_p, P(mhs_host_csr), P(ctypes.c_int64), P(ctypes.c_int64)]
    L.mhs_read_csr_bin.restype = c_int
    L.mhs_flop_count.argtypes = [ctypes.c_int32, c_void_p, c_void_p]
    L.mhs_flop_count.restype = ctypes.c_uint64
    L.mhs_memcpy.argtypes = [c_void_p, c_void_p, c_void_p, c_size_t, c_int]
    L.mhs_memcpy.restype = c_int
    L.mhs_device_alloc.argtypes = [c_void_p, P(c_void_p), c_size_t]
    L.mhs_device_alloc.restype = c_int
    L.mhs_ctx_set_option.argtypes = [c_void_p, c_int, c_int]
    L.mhs_ctx_set_option.restype = c_int
    L.mhs_ctx_numeric_ms.argtypes = [c_void_p, P(ctypes.c_float), c_int]
    L.mhs_ctx_numeric_ms.restype = c_int
    L.mhs_device_free.argtypes = [c_void_p, c_void_p]
    L.mhs_device_free.restype = c_int
    L.mhs_transpose.argtypes = [c_void_p, P(mhs_csr), P(mhs_csr)]
    L.mhs_transpose.restype = c_int
    L.mhs_probe_conflicts.argtypes = [c_void_p, P(ctypes.c_uint64)]
    L.mhs_probe_conflicts.restype = c_int
    L.mhs_ctx_chunked_calls.argtypes = [c_void_p]
    L.mhs_ctx_chunked_calls.restype = ctypes.c_longlong
    if hasattr(L, "mhs_ctx_stat"):  # (ABI 9)
        L.mhs_ctx_stat.argtypes = [c_void_p, c_int]
        L.mhs_ctx_stat.restype = ctypes.c_longlong
    if hasattr(L, "mhs_hbm_peak"):  # (older A/B variant libraries lack the diagnostic)
        L.mhs_hbm_peak.argtypes = [c_void_p, c_size_t, c_int, P(ctypes.c_double)]
        L.mhs_hbm_peak.restype = c_int
    _lib = L
    return L


VENDOR_PATH = HERE / "libmhs_vendor.so"
VENDOR_HEADER = HERE.parent.parent / "include" / "mhs_vendor.h"
_vlib = None


def vendor_lib() -> ctypes.CDLL:
    """libmhs_vendor.so: rocSPARSE SpGEMM, the vendor comparison row (include/mhs_vendor.h)."""
    global _vlib
    if _vlib is not None:
        return _vlib
    lib()  # torch's HIP runtime first (see lib())
    if not VENDOR_PATH.exists():
        raise ImportError(f"{VENDOR_PATH} is missing: build with make -C mh-spgemm_amd")
    V = ctypes.CDLL(str(VENDOR_PATH))
    P = ctypes.POINTER
    V.mhs_vendor_spgemm.argtypes = [ctypes.c_int, P(mhs_csr), P(mhs_csr), P(mhs_csr), P(ctypes.c_double),
                                    ctypes.c_char_p, ctypes.c_int]
    V.mhs_vendor_spgemm.restype = ctypes.c_int
    V.mhs_vendor_free.argtypes = [P(mhs_csr)]
    V.mhs_vendor_free.restype = None
    _vlib = V
    return V


def lib_path() -> str:
    return os.fspath(LIB_PATH)
