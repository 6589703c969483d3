"""Ad-hoc GPU bring-up check (tools only): run the HIP path on a few matrices and diff against the oracle."""
import sys, time
sys.path.insert(0, 'mh-spgemm_amd'); sys.path.insert(0, '.')
import numpy as np
import torch
import mhspgemm as m
from mhspgemm import synth
from oracle import oracle as orc

tool = m.Tool(0)
names = sys.argv[1:] or ["cage4", "cant"]
for name in names:
    A = synth.SYNTH[name]()
    A.H2D(0)
    t0 = time.time()
    C, t = m.spgemm(tool, A, A)
    dt = time.time() - t0
    p, c, v = C.to_host()
    Cp, Ci, Cv = orc.spgemm(A.ptr, A.col, A.val, A.ptr, A.col, A.val, A.N)
    ok = m.compare_tol(Cp, Ci, Cv, p, c, v)
    print(f"{name}: M={A.M} nnzA={A.nnz} nnzC={C.nnz} ref={Cp[-1]} ok={ok} first_call={dt*1e3:.1f}ms", flush=True)
    print("   timing", t, flush=True)
    # timed
    for it in range(3):
        C.release()
        torch.cuda.synchronize()
        t0 = time.time(); C, t = m.spgemm(tool, A, A); dt = time.time() - t0
        print(f"   iter {it}: {dt*1e3:.3f} ms  e2e={t.total_e2e:.3f} ref={t.getTotal():.3f} GFLOPS={2*t.flop/(t.total_e2e*1e6):.1f}", flush=True)
    C.release()
