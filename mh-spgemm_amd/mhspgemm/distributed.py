"""Row-sharded C = A*B over several GPUs of one node.

One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI on
ROCm; "gloo" for CPU tests).  The reference is single-GPU; this is the
north_star's multi-GPU mode:

  1. partition   contiguous A row ranges balanced by flop (products), cut at
                 p*F/P of the int64 prefix sum of per-row flop;
  2. allgatherv  every rank holds its row block of B (B = A for A*A); the
                 blocks (row_ptr, col, val) are exchanged with grouped P2P
                 send/recv straight into place (RCCL has no allgatherv; a
                 padded all_gather would need a compaction copy) and the
                 row_ptr blocks rebased by the nnz prefix;
  3. local       C rows [r_p, r_{p+1}) = A_p * B on each GPU (the HIP library);
  4. gatherv     optional: C's row blocks to rank 0 (grouped P2P, rebased).

C is left distributed by default -- the gather is reported separately (at 8
GPUs its ingress-bound cost can exceed the compute).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np


def row_flop(Aptr: np.ndarray, Acol: np.ndarray, Bptr: np.ndarray) -> np.ndarray:
    """Per-row products of A*B (int64)."""
    blen = np.diff(Bptr.astype(np.int64))
    per = blen[Acol] if len(Acol) else np.zeros(0, np.int64)
    out = np.zeros(len(Aptr) - 1, np.int64)
    rows = np.repeat(np.arange(len(Aptr) - 1), np.diff(Aptr))
    np.add.at(out, rows, per)
    return out


def partition_rows(flop_per_row: np.ndarray, P: int) -> np.ndarray:
    """Boundaries r[0..P] (r[0]=0, r[P]=M): rank p owns [r[p], r[p+1]), cut
    where the inclusive flop prefix first reaches p*F/P."""
    M = len(flop_per_row)
    pre = np.cumsum(flop_per_row.astype(np.int64))
    F = int(pre[-1]) if M else 0
    b = np.zeros(P + 1, np.int64)
    for p in range(1, P):
        if F:
            b[p] = int(np.searchsorted(pre, F * p / P, side="left"))
        else:
            b[p] = (M * p) // P
        b[p] = min(max(b[p], b[p - 1]), M)
    b[P] = M
    return b


@dataclass
class Block:
    """A CSR row block: rows [r0, r1) with a local row_ptr (starting at 0) and
    global column indices; tensors on the rank's device (or CPU for gloo)."""
    r0: int
    r1: int
    ptr: "torch.Tensor"
    col: "torch.Tensor"
    val: "torch.Tensor"


def local_block(ptr: np.ndarray, col: np.ndarray, val: np.ndarray, r0: int, r1: int, device) -> Block:
    import torch
    s, e = int(ptr[r0]), int(ptr[r1])
    p = torch.from_numpy((ptr[r0:r1 + 1].astype(np.int64) - s).astype(np.int32)).to(device)
    return Block(r0, r1, p, torch.from_numpy(np.ascontiguousarray(col[s:e])).to(device),
                 torch.from_numpy(np.ascontiguousarray(val[s:e])).to(device))


def _exchange_sizes(blk: Block, group=None):
    import torch
    import torch.distributed as dist
    P = dist.get_world_size(group)
    dev = blk.col.device
    me = torch.tensor([blk.r1 - blk.r0, blk.col.numel()], dtype=torch.int64, device=dev)
    allv = torch.zeros(P * 2, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(allv, me, group=group)
    a = allv.cpu().numpy().reshape(P, 2)
    return a[:, 0], a[:, 1]


def _p2p_allgatherv(local: "torch.Tensor", out: "torch.Tensor", offs, lens, group=None):
    """Every rank's `local` lands at out[offs[q]:offs[q]+lens[q]] on every rank."""
    import torch.distributed as dist
    P = dist.get_world_size(group)
    me = dist.get_rank(group)
    out[offs[me]:offs[me] + lens[me]].copy_(local)
    ops = []
    for k in range(1, P):  # ring order spreads the pairs over the xGMI links
        dst = (me + k) % P
        src = (me - k) % P
        if lens[me] > 0:
            ops.append(dist.P2POp(dist.isend, local, dst, group))
        if lens[src] > 0:
            ops.append(dist.P2POp(dist.irecv, out[offs[src]:offs[src] + lens[src]], src, group))
    if ops:
        for r in dist.batch_isend_irecv(ops):
            r.wait()


def allgatherv_rows(blk: Block, group=None):
    """allgatherv of CSR row blocks -> full (ptr, col, val) on every rank."""
    import torch
    import torch.distributed as dist
    rows, nnz = _exchange_sizes(blk, group)
    P = len(rows)
    roff = np.concatenate([[0], np.cumsum(rows)])
    noff = np.concatenate([[0], np.cumsum(nnz)])
    dev = blk.col.device
    col = torch.empty(int(noff[-1]), dtype=blk.col.dtype, device=dev)
    val = torch.empty(int(noff[-1]), dtype=blk.val.dtype, device=dev)
    # local row_ptr blocks carry rows+1 entries; exchange the first `rows` of each
    ptr_parts = torch.empty(int(roff[-1]) + 1, dtype=torch.int32, device=dev)
    _p2p_allgatherv(blk.col, col, noff, nnz, group)
    _p2p_allgatherv(blk.val, val, noff, nnz, group)
    _p2p_allgatherv(blk.ptr[:-1].contiguous(), ptr_parts, roff, rows, group)
    # rebase: block q's row pointers += nnz prefix of q
    shift = torch.from_numpy(np.repeat(noff[:-1], rows).astype(np.int32)).to(dev)
    ptr = ptr_parts
    ptr[:-1] += shift
    ptr[-1] = int(noff[-1])
    return ptr, col, val


def gatherv_rows(blk: Block, root: int = 0, group=None):
    """gatherv of CSR row blocks to `root` -> (ptr, col, val) there, None elsewhere."""
    import torch
    import torch.distributed as dist
    rows, nnz = _exchange_sizes(blk, group)
    P = len(rows)
    me = dist.get_rank(group)
    roff = np.concatenate([[0], np.cumsum(rows)])
    noff = np.concatenate([[0], np.cumsum(nnz)])
    dev = blk.col.device
    ops = []
    if me == root:
        col = torch.empty(int(noff[-1]), dtype=blk.col.dtype, device=dev)
        val = torch.empty(int(noff[-1]), dtype=blk.val.dtype, device=dev)
        ptr = torch.empty(int(roff[-1]) + 1, dtype=torch.int32, device=dev)
        col[noff[me]:noff[me + 1]].copy_(blk.col)
        val[noff[me]:noff[me + 1]].copy_(blk.val)
        ptr[roff[me]:roff[me + 1]].copy_(blk.ptr[:-1])
        for q in range(P):
            if q == root:
                continue
            if nnz[q] > 0:
                ops.append(dist.P2POp(dist.irecv, col[noff[q]:noff[q + 1]], q, group))
                ops.append(dist.P2POp(dist.irecv, val[noff[q]:noff[q + 1]], q, group))
            if rows[q] > 0:
                ops.append(dist.P2POp(dist.irecv, ptr[roff[q]:roff[q + 1]], q, group))
    else:
        if nnz[me] > 0:
            ops.append(dist.P2POp(dist.isend, blk.col, root, group))
            ops.append(dist.P2POp(dist.isend, blk.val, root, group))
        if rows[me] > 0:
            ops.append(dist.P2POp(dist.isend, blk.ptr[:-1].contiguous(), root, group))
    if ops:
        for r in dist.batch_isend_irecv(ops):
            r.wait()
    if me != root:
        return None
    shift = torch.from_numpy(np.repeat(noff[:-1], rows).astype(np.int32)).to(dev)
    ptr[:-1] += shift
    ptr[-1] = int(noff[-1])
    return ptr, col, val


def hip_local_multiply(tool):
    """Local multiply on the rank's GPU through the C-ABI: (A block, full B) -> C block."""
    from . import core

    def mult(A: Block, Bptr, Bcol, Bval, N):
        a = core.CSR(A.r1 - A.r0, N)
        a.nnz = A.col.numel()
        a.d_ptr, a.d_col, a.d_val = A.ptr, A.col, A.val
        b = core.CSR(Bptr.numel() - 1, N)
        b.nnz = Bcol.numel()
        b.d_ptr, b.d_col, b.d_val = Bptr, Bcol, Bval
        C, t = core.spgemm(tool, a, b, timing=False)
        return C

    return mult


def spgemm_rowsharded(A_blk: Block, N: int, multiply, group=None, gather: bool = False):
    """Steps 2-4 for this rank: allgatherv(B = A blocks), local multiply,
    optional gatherv of C to rank 0.  Returns (C_local, gathered|None)."""
    Bptr, Bcol, Bval = allgatherv_rows(A_blk, group)
    C = multiply(A_blk, Bptr, Bcol, Bval, N)
    g = None
    if gather:
        g = gather_result(C, A_blk, group)
    return C, g


def gather_result(C, A_blk: Block, group=None):
    """gatherv of a local result (DeviceCSR or (ptr, col, val) tensors) to rank 0."""
    if isinstance(C, tuple):
        p, c, v = C
    else:
        p, c, v = C.to_torch()
    return gatherv_rows(Block(A_blk.r0, A_blk.r1, p, c, v), 0, group)
