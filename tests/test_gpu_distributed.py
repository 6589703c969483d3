"""Row-sharded A*A (BASELINE.json configs[4]) with the HIP library as the local multiply.

Two processes (gloo rendezvous on 127.0.0.1) share the one GPU of the test box: the
flop balance (`rebalance`) and the exchange plan (`ShardPlan`) run on CPU tensors over
gloo exactly as they do over RCCL; each rank then moves its renumbered A block and the
exchanged B rows to cuda:0 and calls `hip_local_multiply` -- `mhs_spgemm` through the
C-ABI on an A whose columns index a rectangular local B (nB rows x M_global columns),
the shape no single-process test exercises.  C's row blocks come back with gatherv and
rank 0 compares the whole product with the oracle: row_ptr and col_idx bit-exact,
values within 1e-6 relative (the reference's MH_spgemm on the rank's rows,
/root/reference/src/main.cu:12-72).
"""
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parent.parent


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _matrix(kind):
    from mhspgemm import synth
    if kind == "banded":  # 200 k rows, +-1000 band, no long-range columns: a halo exchange
        return synth.banded_random(200_000, 12.0, 1000, far_frac=0.0, seed=21)
    # cage15-like structure (synth.cage15_like's generator) at 300 k rows: 10 % of the
    # columns anywhere, so every rank needs rows of every other rank
    return synth.banded_random(300_000, 18.2, 300, far_frac=0.10, seed=7)


def _worker(rank, world, port, q, kind, mode):
    try:
        sys.path[:0] = [str(ROOT), str(ROOT / "mh-spgemm_amd"), str(ROOT / "tests")]
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                          WORLD_SIZE=str(world))
        import torch
        import torch.distributed as dist
        import mhspgemm
        from mhspgemm import distributed as D

        dist.init_process_group("gloo", rank=rank, world_size=world)
        A = _matrix(kind)
        r0, r1 = D.equal_rows(A.M, world, rank)
        eq = D.local_block(A.ptr, A.col, A.val, r0, r1, "cpu")
        blk = D.rebalance(eq, A.M)
        plan = D.ShardPlan(blk, A.M, mode=mode)
        tool = mhspgemm.Tool(0)
        mult = D.hip_local_multiply(tool)
        la = plan.local_A()
        la_gpu = D.Block(la.r0, la.r1, la.ptr.to("cuda:0"), la.col.to("cuda:0"), la.val.to("cuda:0"))
        for step in range(2):  # the plan is reused across steps
            Bp, Bc, Bv = plan.exchange()
            C = mult(la_gpu, Bp.to("cuda:0"), Bc.to("cuda:0"), Bv.to("cuda:0"), A.M)
            p, c, v = (x.cpu() for x in C.to_torch())
            C.release()
            g = D.gather_result((p, c, v), blk)
        tool.close()
        res = {"rank": rank, "nB": plan.nB, "rows": (blk.r0, blk.r1), "B_rect": (plan.nB, A.M)}
        if rank == 0:
            from oracle import oracle as orc
            Cp, Ci, Cv = orc.spgemm(A.ptr, A.col, A.val, A.ptr, A.col, A.val, A.N)
            gp, gc, gv = (x.numpy() for x in g)
            res["ptr_ok"] = bool(np.array_equal(gp, Cp))
            res["col_ok"] = bool(res["ptr_ok"] and np.array_equal(gc, Ci))
            ok, *_ = mhspgemm.compare_tol(Cp, Ci, Cv, gp, gc, gv, 1e-6, 1e-12)
            res["val_ok"] = bool(ok)
            res["nnzC"] = int(Cp[-1])
        dist.barrier()
        dist.destroy_process_group()
        q.put(res)
    except Exception:
        import traceback
        q.put({"rank": rank, "error": traceback.format_exc()})


@pytest.mark.parametrize("kind,mode", [("banded", "halo"), ("cage15-block", "halo"), ("cage15-block", "full")])
def test_rowsharded_hip_local_multiply(kind, mode):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, kind, mode)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        out = [q.get(timeout=240) for _ in range(world)]
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    errs = [o["error"] for o in out if "error" in o]
    assert not errs, errs[0]
    r0 = next(o for o in out if o["rank"] == 0)
    assert r0["ptr_ok"] and r0["col_ok"], r0
    assert r0["val_ok"], r0
    rows = sorted(o["rows"] for o in out)
    assert rows[0][0] == 0 and rows[0][1] == rows[1][0]
    if mode == "halo" and kind == "banded":  # each rank's local B is its halo, not the whole matrix
        assert all(o["nB"] < 200_000 for o in out), out
    print(kind, mode, [o.get("B_rect") for o in out], r0["nnzC"])
