"""mhspgemm -- MI355X-native mask-and-hash SpGEMM (C = A*B, CSR, FP64).

Host-side mirror of the reference yyssys/MH-SpGEMM driver surface over the
C-ABI of libmhspgemm.so (include/mhspgemm.h).  The compute path is the HIP
library only; importing this package without the built library raises.
"""
from ._lib import lib, lib_path, declared_functions, MHS_OK  # noqa: F401
from .core import (CSR, DeviceCSR, MHSpGEMMError, MH_spgemm, Timing, Tool, compare_ref,  # noqa: F401
                   compare_tol, flop_count, flop_count_np, matrix_transposition, readMtxFile, spgemm,
                   transpose, vendor_spgemm)

lib()  # fail loudly at import if the HIP extension is missing

__all__ = ["CSR", "DeviceCSR", "MHSpGEMMError", "MH_spgemm", "Timing", "Tool", "compare_ref",
           "compare_tol", "flop_count", "flop_count_np", "matrix_transposition", "readMtxFile", "spgemm",
           "transpose", "vendor_spgemm", "lib"]
