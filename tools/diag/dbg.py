import sys, os; os.environ.setdefault("MHS_LIB", "tools/diag/vdbg/libmhspgemm.so"); sys.path[:0]=[".", "mh-spgemm_amd", "tests"]
import numpy as np, torch, mhspgemm
from oracle import oracle as orc
from _util import GOLDEN
A = mhspgemm.CSR(); mhspgemm.readMtxFile(A, str(GOLDEN / "cage4_like_A.mtx"))
print("A ptr", A.ptr.tolist()); print("A col", A.col.tolist())
t = mhspgemm.Tool(0); A.H2D(0)
C, tm = mhspgemm.spgemm(t, A, A); p, c, v = C.to_host()
Cp, Ci, Cv = orc.spgemm(A.ptr, A.col, A.val, A.ptr, A.col, A.val, A.N)
print("bins", tm.num_bins[:8], tm.sym_bins[:5])
for i in range(A.M):
    d = np.abs(v[p[i]:p[i+1]] - Cv[Cp[i]:Cp[i+1]]) / np.abs(Cv[Cp[i]:Cp[i+1]])
    print(i, "maxrel", d.max() if len(d) else 0, "ratio", (v[p[i]:p[i+1]] / Cv[Cp[i]:Cp[i+1]])[:4])
