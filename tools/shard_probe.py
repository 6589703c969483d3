"""Single-GPU rehearsal of the row-sharded step: for P in 1,2,4,8, the local
SpGEMM of every rank's block against its halo B (what ShardPlan's halo mode
hands the HIP library), timed one rank at a time on this GPU; prints the max
over ranks (the step's compute bound) and the halo bytes a rank would receive.
usage: python tools/shard_probe.py [matrix]"""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "mh-spgemm_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import mhspgemm  # noqa: E402
from mhspgemm import synth, distributed as D, _lib as L  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "cant"
A, _ = synth.load_or_synth(name)
flop = mhspgemm.flop_count_np(A.col, A.ptr)
tool = mhspgemm.Tool(0)
tool.set_stream(torch.cuda.current_stream(0).cuda_stream)
rf = D.row_flop(A.ptr, A.col, A.ptr)
for P in (1, 2, 4, 8):
    bnd = D.partition_rows(rf, P)
    worst, xb = 0.0, 0
    for p in range(P):
        r0, r1 = int(bnd[p]), int(bnd[p + 1])
        s, e = int(A.ptr[r0]), int(A.ptr[r1])
        lcol = A.col[s:e]
        need = np.unique(lcol)
        pos = np.searchsorted(need, lcol).astype(np.int32)
        lens = np.diff(A.ptr)[need]
        Bp = np.zeros(len(need) + 1, np.int64)
        Bp[1:] = np.cumsum(lens)
        sel = np.concatenate([np.arange(A.ptr[r], A.ptr[r + 1]) for r in need])
        a = mhspgemm.CSR(r1 - r0, len(need), (A.ptr[r0:r1 + 1] - s).astype(np.int32), pos, A.val[s:e])
        b = mhspgemm.CSR(len(need), A.N, Bp.astype(np.int32), A.col[sel], A.val[sel])
        a.H2D(0)
        b.H2D(0)
        remote = (need < r0) | (need >= r1)
        xb = max(xb, int(4 * remote.sum() + 12 * lens[remote].sum()))
        tool.set_option(L.MHS_OPT_SYNC, 0)
        for _ in range(3):
            C, _ = mhspgemm.spgemm(tool, a, b, timing=False)
            C.release()
        torch.cuda.synchronize()
        t0 = torch.cuda.Event(enable_timing=True)
        t1 = torch.cuda.Event(enable_timing=True)
        import time
        h0 = time.perf_counter()
        for _ in range(10):
            C, _ = mhspgemm.spgemm(tool, a, b, timing=False)
            C.release()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - h0) / 10 * 1e3
        worst = max(worst, ms)
    print(json.dumps({"matrix": name, "P": P, "max_rank_ms": round(worst, 4),
                      "gflops_if_exchange_free": round(2 * flop / (worst * 1e-3) / 1e9, 1),
                      "max_halo_bytes_in": xb}), flush=True)
