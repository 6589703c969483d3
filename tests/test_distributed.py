"""Row-sharded multi-process path (mhspgemm.distributed) on CPU with gloo.

World size 2 (and 3 for uneven shards), 127.0.0.1 rendezvous.  The exchange
steps (flop-balanced partition, allgatherv of B's row blocks, gatherv of C's
row blocks) are the product code; the local multiply is injected -- on the GPU
it is the HIP library, here the oracle (test infrastructure) so the exchange
logic is checked bit-exactly without a GPU.
"""
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parent.parent


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _matrix(seed=3, M=700, per=6):
    rng = np.random.default_rng(seed)
    lens = rng.poisson(per, M)
    lens[::17] = 0  # empty rows
    rows = np.repeat(np.arange(M), lens)
    cols = rng.integers(0, M, len(rows))
    key = np.unique(rows.astype(np.int64) * M + cols)
    r = key // M
    c = (key % M).astype(np.int32)
    ptr = np.zeros(M + 1, np.int64)
    np.cumsum(np.bincount(r, minlength=M), out=ptr[1:])
    return M, ptr.astype(np.int32), c, rng.uniform(0.1, 1.0, len(c))


def _worker(rank, world, port, q):
    try:
        sys.path[:0] = [str(ROOT), str(ROOT / "mh-spgemm_amd"), str(ROOT / "tests")]
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                          WORLD_SIZE=str(world))
        import torch
        import torch.distributed as dist
        from mhspgemm import distributed as D
        from oracle import oracle as orc

        dist.init_process_group("gloo", rank=rank, world_size=world)
        M, ptr, col, val = _matrix()
        rf = D.row_flop(ptr, col, ptr)
        bnd = D.partition_rows(rf, world)
        blk = D.local_block(ptr, col, val, int(bnd[rank]), int(bnd[rank + 1]), "cpu")

        # allgatherv(B): every rank must hold the whole matrix
        Bp, Bc, Bv = D.allgatherv_rows(blk)
        ok_b = (np.array_equal(Bp.numpy(), ptr) and np.array_equal(Bc.numpy(), col)
                and np.array_equal(Bv.numpy(), val))

        def mult(A, Bptr, Bcol, Bval, N):
            Cp, Ci, Cv = orc.spgemm(A.ptr.numpy(), A.col.numpy(), A.val.numpy(), Bptr.numpy(),
                                    Bcol.numpy(), Bval.numpy(), N)
            return torch.from_numpy(Cp), torch.from_numpy(Ci), torch.from_numpy(Cv)

        C, g = D.spgemm_rowsharded(blk, M, mult, gather=True)
        res = {"rank": rank, "ok_b": ok_b, "rows": (int(bnd[rank]), int(bnd[rank + 1])),
               "flop": int(rf[bnd[rank]:bnd[rank + 1]].sum())}
        if rank == 0:
            Cp, Ci, Cv = orc.spgemm(ptr, col, val, ptr, col, val, M)
            gp, gc, gv = (x.numpy() for x in g)
            res["ok_c"] = (np.array_equal(gp, Cp) and np.array_equal(gc, Ci) and np.array_equal(gv, Cv))
            res["bnd"] = bnd.tolist()
        dist.barrier()
        dist.destroy_process_group()
        q.put(res)
    except Exception as e:  # surface worker failures in the parent
        import traceback
        q.put({"rank": rank, "error": traceback.format_exc()})


def _planned_worker(rank, world, port, q, mode, order="ranked"):
    try:
        sys.path[:0] = [str(ROOT), str(ROOT / "mh-spgemm_amd"), str(ROOT / "tests")]
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                          WORLD_SIZE=str(world))
        import torch
        import torch.distributed as dist
        from mhspgemm import distributed as D
        from oracle import oracle as orc

        dist.init_process_group("gloo", rank=rank, world_size=world)
        M, ptr, col, val = _banded(M=900)
        rf = D.row_flop(ptr, col, ptr)
        bnd = D.partition_rows(rf, world)
        q_ = world - 1 - rank if order == "reversed" else rank  # "reversed": ranges not in rank order
        blk = D.local_block(ptr, col, val, int(bnd[q_]), int(bnd[q_ + 1]), "cpu")
        if order == "gap":  # rank 0 owns no rows at the front: not a tiling
            blk = D.local_block(ptr, col, val, int(bnd[q_]) + (5 if rank == 0 else 0), int(bnd[q_ + 1]), "cpu")
        if order != "ranked":  # blocks that do not tile [0, M) in rank order are refused on every rank
            try:
                D.ShardPlan(blk, M, mode=mode)
                ok = False
            except ValueError:
                ok = True
            dist.destroy_process_group()
            q.put({"rank": rank, "ok_b": ok, "ok_c": ok, "nB": 0})
            return
        plan = D.ShardPlan(blk, M, mode=mode)
        # the local B holds exactly the planned rows of the global matrix
        Bp, Bc, Bv = plan.exchange()
        rows = plan.brows
        exp_len = np.diff(ptr)[rows]
        ok_b = np.array_equal(np.diff(Bp.numpy()), exp_len)
        sel = np.concatenate([np.arange(ptr[r], ptr[r + 1]) for r in rows]) if len(rows) else np.zeros(0, int)
        ok_b = ok_b and np.array_equal(Bc.numpy(), col[sel]) and np.array_equal(Bv.numpy(), val[sel])
        if mode == "halo":  # a banded matrix needs far fewer than all rows on every rank
            ok_b = ok_b and plan.nB < M

        def mult(A, Bptr, Bcol, Bval, N):
            Cp, Ci, Cv = orc.spgemm(A.ptr.numpy(), A.col.numpy(), A.val.numpy(), Bptr.numpy(),
                                    Bcol.numpy(), Bval.numpy(), N)
            return torch.from_numpy(Cp), torch.from_numpy(Ci), torch.from_numpy(Cv)

        for _ in range(2):  # the plan is reused across steps
            C, g = D.spgemm_planned(plan, mult, gather=True)
        res = {"rank": rank, "ok_b": bool(ok_b), "nB": plan.nB}
        if rank == 0:
            Cp, Ci, Cv = orc.spgemm(ptr, col, val, ptr, col, val, M)
            gp, gc, gv = (x.numpy() for x in g)
            res["ok_c"] = (np.array_equal(gp, Cp) and np.array_equal(gc, Ci) and np.array_equal(gv, Cv))
        dist.barrier()
        dist.destroy_process_group()
        q.put(res)
    except Exception:
        import traceback
        q.put({"rank": rank, "error": traceback.format_exc()})


def _banded(M=900, width=40, per=8, seed=4):
    rng = np.random.default_rng(seed)
    rows = np.repeat(np.arange(M), per)
    cols = np.clip(rows + rng.integers(-width, width + 1, len(rows)), 0, M - 1)
    key = np.unique(rows.astype(np.int64) * M + cols)
    r, c = key // M, (key % M).astype(np.int32)
    ptr = np.zeros(M + 1, np.int64)
    np.cumsum(np.bincount(r, minlength=M), out=ptr[1:])
    return M, ptr.astype(np.int32), c, rng.uniform(0.1, 1.0, len(c))


@pytest.mark.parametrize("world,mode,order", [(2, "halo", "ranked"), (3, "halo", "ranked"), (3, "full", "ranked"),
                                              (4, "halo", "ranked"), (4, "full", "ranked"), (3, "full", "reversed"),
                                              (3, "full", "gap")])
def test_planned_exchange_gloo(world, mode, order):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_planned_worker, args=(r, world, port, q, mode, order)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    errs = [o["error"] for o in out if "error" in o]
    assert not errs, errs[0]
    assert all(o["ok_b"] for o in out), out
    assert next(o for o in out if o["rank"] == 0)["ok_c"], "gatherv(C) must equal the single-process product"


@pytest.mark.parametrize("world", [2, 3])
def test_rowsharded_allgatherv_gatherv_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    errs = [o["error"] for o in out if "error" in o]
    assert not errs, errs[0]
    assert all(o["ok_b"] for o in out), "allgatherv(B) must reassemble A exactly on every rank"
    r0 = next(o for o in out if o["rank"] == 0)
    assert r0["ok_c"], "gatherv(C) must equal the single-process product bit-exactly"
    # contiguous cover of the rows
    rows = sorted(o["rows"] for o in out)
    assert rows[0][0] == 0 and all(rows[i][1] == rows[i + 1][0] for i in range(world - 1))


def _rebalance_worker(rank, world, port, q):
    try:
        sys.path[:0] = [str(ROOT), str(ROOT / "mh-spgemm_amd"), str(ROOT / "tests")]
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                          WORLD_SIZE=str(world))
        import torch.distributed as dist
        from mhspgemm import distributed as D

        dist.init_process_group("gloo", rank=rank, world_size=world)
        res = {"rank": rank}
        for seed in (3, 8):
            M, ptr, col, val = _matrix(seed=seed, M=1500)
            if seed == 8:  # two dense rows hold most of the flop: cuts land on or next to them
                dense = {100: np.arange(M, dtype=np.int32), 101: np.arange(0, M, 2, dtype=np.int32)}
                rows = [dense.get(i, col[ptr[i]:ptr[i + 1]]) for i in range(M)]
                ptr = np.concatenate([[0], np.cumsum([len(r) for r in rows])]).astype(np.int32)
                col = np.concatenate(rows).astype(np.int32)
                val = np.linspace(0.1, 1.0, len(col))
            r0, r1 = D.equal_rows(M, world, rank)
            eq = D.local_block(ptr, col, val, r0, r1, "cpu")
            nb = D.rebalance(eq, M)
            bnd = D.partition_rows(D.row_flop(ptr, col, ptr), world)
            ref = D.local_block(ptr, col, val, int(bnd[rank]), int(bnd[rank + 1]), "cpu")
            res[f"ok{seed}"] = bool((nb.r0, nb.r1) == (ref.r0, ref.r1) and np.array_equal(nb.ptr.numpy(), ref.ptr.numpy())
                                    and np.array_equal(nb.col.numpy(), ref.col.numpy())
                                    and np.array_equal(nb.val.numpy(), ref.val.numpy()))
        dist.barrier()
        dist.destroy_process_group()
        q.put(res)
    except Exception:
        import traceback
        q.put({"rank": rank, "error": traceback.format_exc()})


@pytest.mark.parametrize("world", [2, 3, 4])
def test_rebalance_matches_partition_gloo(world):
    # the distributed flop balance (each rank starts from an equal-row block, never the
    # whole matrix) gives every rank exactly the block partition_rows assigns it
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rebalance_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    errs = [o["error"] for o in out if "error" in o]
    assert not errs, errs[0]
    assert all(o["ok3"] and o["ok8"] for o in out), out


def test_partition_balances_flop():
    from mhspgemm import distributed as D
    rng = np.random.default_rng(0)
    f = rng.integers(0, 100, 10_000)
    f[5000:5010] = 50_000  # heavy rows
    for P in (1, 2, 4, 8):
        b = D.partition_rows(f, P)
        assert b[0] == 0 and b[-1] == len(f) and np.all(np.diff(b) >= 0)
        parts = [f[b[p]:b[p + 1]].sum() for p in range(P)]
        assert max(parts) <= f.sum() / P + f.max()  # within one row of the ideal cut
    b = D.partition_rows(np.zeros(10, np.int64), 4)
    assert b.tolist() == [0, 2, 5, 7, 10]


def test_row_flop_matches_oracle():
    from mhspgemm import distributed as D
    from oracle import oracle as orc
    M, ptr, col, val = _matrix(seed=5)
    rf = D.row_flop(ptr, col, ptr)
    assert rf.sum() == orc.flop(col, ptr)
