"""Row-sharded C = A*B over several GPUs of one node.

One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI on
ROCm; "gloo" for CPU tests).  The reference is single-GPU; this is the
north_star's multi-GPU mode:

  1. partition   contiguous A row ranges balanced by flop (products), cut at
                 p*F/P of the int64 prefix sum of per-row flop -- `rebalance`
                 computes the cuts from the ranks' own (equal-row) blocks plus
                 the all-gathered row lengths and moves rows to their owners,
                 so no rank needs the whole matrix;
  2. exchange    every rank holds its row block of B (B = A for A*A) and needs
                 the B rows its A block references.  Two executors of one plan:
                 * "halo" (default): a rank receives only the rows its columns
                   name -- the allgatherv restricted to the referenced rows (for
                   banded / FEM matrices a halo of the neighbours' rows);
                 * "full": the north_star's allgatherv of every row block.
                 The plan (which rows go where, receive offsets, A's columns
                 renumbered to local B rows) is built once by `ShardPlan` with
                 one all_gather + two all_to_all of counts and row lists; every
                 step then moves the rows' lengths, columns and values with
                 grouped P2P send/recv straight into place (RCCL has no
                 allgatherv) and rebuilds B's row pointer with one cumsum -- no
                 host round trip inside a step;
  3. local       C rows [r_p, r_{p+1}) = A_p * B_p on each GPU (the HIP library);
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
    # np.array copies: the inputs may be read-only memory maps (bench.py's shared host copy)
    return Block(r0, r1, p, torch.from_numpy(np.array(col[s:e], dtype=np.int32)).to(device),
                 torch.from_numpy(np.array(val[s:e], dtype=np.float64)).to(device))


def equal_rows(M: int, P: int, p: int):
    """Rows [M*p/P, M*(p+1)/P): the block a rank loads before the flop balance."""
    return (M * p) // P, (M * (p + 1)) // P


def rebalance(blk: Block, M_global: int, group=None, compute=None) -> Block:
    """Distributed flop-balanced partition: from any contiguous row blocks (e.g. the
    equal-row blocks each rank read), compute the cuts of `partition_rows` over the
    global per-row flop without any rank holding the whole matrix, then move rows to
    their new owners.  Traffic: the global row lengths (4 B per row, all-gathered: the
    flop of a row needs the lengths of the B rows it names) plus the rows that change
    owner.  Returns this rank's new block (same contents as `local_block` of the cuts).
    `compute`: device of the per-row flop gathers when the block lives elsewhere (a gloo
    rehearsal keeps the block on the host but computes on the GPU)."""
    import torch
    import torch.distributed as dist
    P = dist.get_world_size(group)
    me = dist.get_rank(group)
    dev = blk.col.device
    rows, _ = _exchange_sizes(blk, group)
    roff = np.concatenate([[0], np.cumsum(rows)])
    assert roff[-1] == M_global, "blocks must cover the rows"
    # 1. global row lengths
    lens = (blk.ptr[1:] - blk.ptr[:-1]).to(torch.int32)
    glen = torch.empty(M_global, dtype=torch.int32, device=dev)
    _p2p_allgatherv(lens, glen, roff, rows, group)
    # 2. local per-row flop, inclusive prefix, per-rank totals
    nloc = blk.r1 - blk.r0
    # (row sums as differences of one prefix over the entries: no per-entry row ids)
    cdev = compute if compute is not None else dev
    per = glen.to(cdev).index_select(0, blk.col.to(cdev).long()).to(torch.int64)
    cs = torch.zeros(per.numel() + 1, dtype=torch.int64, device=cdev)
    torch.cumsum(per, 0, out=cs[1:])
    pre = (cs.index_select(0, blk.ptr[1:].to(cdev).long()) - cs[int(blk.ptr[0])]).to(dev)
    del per, cs
    tot = torch.tensor([int(pre[-1]) if nloc else 0], dtype=torch.int64, device=dev)
    tots = torch.zeros(P, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(tots, tot, group=group)
    tots = tots.cpu().numpy()
    off = int(tots[:me].sum())
    F = int(tots.sum())
    # 3. the cuts falling in this rank's prefix range (partition_rows' rule), max-reduced
    cut = np.zeros(P + 1, np.int64)
    if F and nloc:
        gpre = pre.cpu().numpy() + off
        for q in range(1, P):
            tgt = F * q / P
            if off < tgt <= gpre[-1]:
                cut[q] = blk.r0 + int(np.searchsorted(gpre, tgt, side="left"))
    cut_t = torch.from_numpy(cut).to(dev)
    dist.all_reduce(cut_t, op=dist.ReduceOp.MAX, group=group)
    b = cut_t.cpu().numpy()
    for q in range(1, P):
        if not F:
            b[q] = (M_global * q) // P
        b[q] = min(max(b[q], b[q - 1]), M_global)
    b[0], b[P] = 0, M_global
    # 4. move rows: my [r0, r1) ∩ [b[q], b[q+1]) goes to q, in row order
    lptr = blk.ptr.cpu().numpy().astype(np.int64)
    srow = [max(0, min(blk.r1, int(b[q + 1])) - max(blk.r0, int(b[q]))) for q in range(P)]
    sfirst = [min(max(blk.r0, int(b[q])), blk.r1) - blk.r0 for q in range(P)]
    snnz = [int(lptr[sfirst[q] + srow[q]] - lptr[sfirst[q]]) if srow[q] else 0 for q in range(P)]
    cnt = torch.tensor(srow + snnz, dtype=torch.int64, device=dev).view(2, P).t().contiguous().view(-1)
    cnt_in = torch.zeros(2 * P, dtype=torch.int64, device=dev)
    dist.all_to_all_single(cnt_in, cnt, group=group)
    cin = cnt_in.cpu().numpy().reshape(P, 2)
    rrow, rnnz = cin[:, 0], cin[:, 1]
    nr, nn = int(b[me + 1] - b[me]), int(rnnz.sum())
    assert int(rrow.sum()) == nr
    olen = torch.empty(nr, dtype=torch.int32, device=dev)
    ocol = torch.empty(nn, dtype=blk.col.dtype, device=dev)
    oval = torch.empty(nn, dtype=blk.val.dtype, device=dev)
    ro = np.concatenate([[0], np.cumsum(rrow)])
    no = np.concatenate([[0], np.cumsum(rnnz)])
    ops = []
    for k in range(P):  # self first (a copy), then ring order
        q_dst, q_src = (me + k) % P, (me - k) % P
        a0 = sfirst[q_dst]
        e0 = int(lptr[a0])
        if q_dst == me:
            if srow[me]:
                olen[ro[me]:ro[me + 1]].copy_(lens[a0:a0 + srow[me]])
                ocol[no[me]:no[me + 1]].copy_(blk.col[e0:e0 + snnz[me]])
                oval[no[me]:no[me + 1]].copy_(blk.val[e0:e0 + snnz[me]])
            continue
        if srow[q_dst]:
            ops.append(dist.P2POp(dist.isend, lens[a0:a0 + srow[q_dst]].contiguous(), q_dst, group))
        if snnz[q_dst]:
            ops.append(dist.P2POp(dist.isend, blk.col[e0:e0 + snnz[q_dst]].contiguous(), q_dst, group))
            ops.append(dist.P2POp(dist.isend, blk.val[e0:e0 + snnz[q_dst]].contiguous(), q_dst, group))
        if rrow[q_src]:
            ops.append(dist.P2POp(dist.irecv, olen[ro[q_src]:ro[q_src + 1]], q_src, group))
        if rnnz[q_src]:
            ops.append(dist.P2POp(dist.irecv, ocol[no[q_src]:no[q_src + 1]], q_src, group))
            ops.append(dist.P2POp(dist.irecv, oval[no[q_src]:no[q_src + 1]], q_src, group))
    if ops:
        for r in dist.batch_isend_irecv(ops):
            r.wait()
    optr = torch.zeros(nr + 1, dtype=torch.int32, device=dev)
    torch.cumsum(olen, 0, out=optr[1:])
    return Block(int(b[me]), int(b[me + 1]), optr, ocol, oval)


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
        a = core.CSR(A.r1 - A.r0, Bptr.numel() - 1)  # A's columns index the local B rows
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


# ------------------------------------------------------------ planned exchange ---

class ShardPlan:
    """Inspector/executor exchange of B's rows for a row-sharded A*B (B = A).

    Built once from this rank's block (collectives over `group`); `exchange()`
    then moves the rows every step.  mode "halo": only the B rows the block's
    columns reference; "full": every row (the north_star's allgatherv).  The
    local B keeps rows in ascending global order (owners' ranges are ascending
    and each request list is sorted), so consecutive rows stay consecutive (FEM
    dof runs) and A's renumbered columns stay sorted per row.

    Round 5: the plan is built with torch ops on the block's device (the GPU under
    RCCL) instead of host numpy -- the round-4 build took 4.9 s at N = 2 on
    cage15-like, most of it np.searchsorted / np.repeat over the block's 50 M
    columns -- and the full mode needs no index lists at all: every peer receives
    the sender's whole block, so a step sends the block's own arrays and A's
    columns are already local B ids."""

    def __init__(self, blk: Block, M_global: int, group=None, mode: str = "halo"):
        import torch
        import torch.distributed as dist
        assert mode in ("halo", "full")
        self.blk, self.mode, self.group = blk, mode, group
        P = dist.get_world_size(group)
        me = dist.get_rank(group)
        self.P, self.me = P, me
        dev = blk.col.device
        self.dev = dev
        # 1. row ranges and nnz of every rank
        rr = torch.tensor([blk.r0, blk.r1, blk.col.numel()], dtype=torch.int64, device=dev)
        allr = torch.zeros(3 * P, dtype=torch.int64, device=dev)
        dist.all_gather_into_tensor(allr, rr, group=group)
        rng = allr.cpu().numpy().reshape(P, 3)
        self.ranges = rng[:, :2]
        self.rowlen = (blk.ptr[1:] - blk.ptr[:-1]).to(torch.int32)
        nrow, nnz = blk.r1 - blk.r0, blk.col.numel()
        # B = A is held as the ranks' row blocks: they must tile [0, M_global) in rank order (the full
        # mode stacks them as B and reads A's global columns as local B ids; the halo mode finds a
        # row's owner by searching the range starts).  Every rank sees the same ranges, so either
        # all raise or none (the check had gone with the round-5 full-mode rewrite)
        if not (rng[0, 0] == 0 and rng[-1, 1] == M_global and all(rng[:, 1] >= rng[:, 0]) and
                all(rng[q, 1] == rng[q + 1, 0] for q in range(P - 1))):
            raise ValueError("ShardPlan: the ranks' row blocks must tile [0, M) in rank order")
        if mode == "full":
            # every peer gets this rank's whole block; this rank gets every block
            self.srows = [nrow] * P
            self.snnz = [nnz] * P
            self.rrows = [int(rng[q, 1] - rng[q, 0]) for q in range(P)]
            self.rnnz = [int(rng[q, 2]) for q in range(P)]
            self.sidx_rows = self.sidx_elems = None
            self.acol_local = blk.col  # B holds every row in order: global ids are local ids
            self._brows_t = None
        else:
            # 2. rows this rank needs from every owner (sorted, global ids), split by owner
            u = torch.unique(blk.col.to(torch.int64))  # sorted
            starts = torch.from_numpy(np.ascontiguousarray(rng[:, 0])).to(dev)
            cut = torch.searchsorted(u, starts).cpu().numpy().tolist() + [u.numel()]
            cnt = [cut[q + 1] - cut[q] for q in range(P)]
            cnt_t = torch.tensor(cnt, dtype=torch.int64, device=dev)
            cnt_in_t = torch.zeros(P, dtype=torch.int64, device=dev)
            dist.all_to_all_single(cnt_in_t, cnt_t, group=group)
            cnt_in = cnt_in_t.cpu().numpy().tolist()
            req_in = torch.zeros(int(sum(cnt_in)), dtype=torch.int64, device=dev)
            dist.all_to_all_single(req_in, u, output_split_sizes=cnt_in, input_split_sizes=cnt, group=group)
            # 3. what this rank sends: rows (local ids) and their entries, per peer
            rows = req_in - blk.r0
            lens = self.rowlen.index_select(0, rows).to(torch.int64)
            rb = blk.ptr.index_select(0, rows).to(torch.int64)
            tot = int(lens.sum()) if lens.numel() else 0
            first = torch.cumsum(lens, 0) - lens
            self.sidx_elems = (torch.repeat_interleave(rb - first, lens) +
                               torch.arange(tot, dtype=torch.int64, device=dev))
            self.sidx_rows = rows
            seg = np.concatenate([[0], np.cumsum(cnt_in)]).astype(np.int64)
            cl = torch.cumsum(lens, 0).cpu().numpy() if lens.numel() else np.zeros(0, np.int64)
            ends = [int(cl[seg[q + 1] - 1]) if seg[q + 1] > 0 else 0 for q in range(P)]
            send_nnz = [ends[q] - (ends[q - 1] if q else 0) for q in range(P)]
            nnz_out = torch.tensor(send_nnz, dtype=torch.int64, device=dev)
            nnz_in = torch.zeros(P, dtype=torch.int64, device=dev)
            dist.all_to_all_single(nnz_in, nnz_out, group=group)
            self.srows = cnt_in
            self.snnz = send_nnz
            self.rrows = cnt
            self.rnnz = [int(x) for x in nnz_in.cpu().numpy()]
            # 4. local B rows = u (ascending global ids); A's columns renumbered into them
            self._brows_t = u
            self.acol_local = torch.searchsorted(u, blk.col.to(torch.int64)).to(torch.int32)
        self.soff_r = np.concatenate([[0], np.cumsum(self.srows)]).astype(np.int64)
        self.soff_n = np.concatenate([[0], np.cumsum(self.snnz)]).astype(np.int64)
        self.roff_r = np.concatenate([[0], np.cumsum(self.rrows)]).astype(np.int64)
        self.roff_n = np.concatenate([[0], np.cumsum(self.rnnz)]).astype(np.int64)
        self.nB = int(self.roff_r[-1])
        self.Bnnz = int(self.roff_n[-1])
        self.M_global = M_global
        # receive buffers (reused every step)
        self.Blen = torch.empty(self.nB, dtype=torch.int32, device=dev)
        self.Bcol = torch.empty(self.Bnnz, dtype=blk.col.dtype, device=dev)
        self.Bval = torch.empty(self.Bnnz, dtype=blk.val.dtype, device=dev)
        self.Bptr = torch.zeros(self.nB + 1, dtype=torch.int32, device=dev)
        self.bytes_in = 4 * self.nB + 12 * self.Bnnz - (4 * self.rrows[me] + 12 * self.rnnz[me])

    @property
    def brows(self) -> np.ndarray:
        """Global ids of the local B rows (ascending)."""
        if self._brows_t is None:
            return np.arange(self.M_global, dtype=np.int64)
        return self._brows_t.cpu().numpy()

    def _packed(self):
        """(row lengths, columns, values) to send, concatenated over peers in rank order
        (full mode: the block itself, the same slice for every peer)."""
        blk = self.blk
        if self.sidx_rows is None:
            return self.rowlen, blk.col, blk.val
        return (self.rowlen.index_select(0, self.sidx_rows), blk.col.index_select(0, self.sidx_elems),
                blk.val.index_select(0, self.sidx_elems))

    def exchange(self):
        """One step: pack the requested rows, P2P them into place, rebuild B's row
        pointer.  Returns (Bptr, Bcol, Bval) over the local B rows."""
        import torch
        import torch.distributed as dist
        me, P = self.me, self.P
        full = self.sidx_rows is None
        sl, sc, sv = self._packed()

        def out_slice(q):  # this rank's send slice for peer q
            if full:
                return (0, self.srows[q]), (0, self.snnz[q])
            return (self.soff_r[q], self.soff_r[q + 1]), (self.soff_n[q], self.soff_n[q + 1])

        (s0, s1), (e0, e1) = out_slice(me)
        r0, r1 = self.roff_r[me], self.roff_r[me + 1]
        n0, n1 = self.roff_n[me], self.roff_n[me + 1]
        self.Blen[r0:r1].copy_(sl[s0:s1])
        self.Bcol[n0:n1].copy_(sc[e0:e1])
        self.Bval[n0:n1].copy_(sv[e0:e1])
        ops = []
        for k in range(1, P):  # ring order spreads the pairs over the xGMI links
            dst, src = (me + k) % P, (me - k) % P
            (a, b), (c, d) = out_slice(dst)
            if self.srows[dst]:
                ops.append(dist.P2POp(dist.isend, sl[a:b], dst, self.group))
            if self.snnz[dst]:
                ops.append(dist.P2POp(dist.isend, sc[c:d], dst, self.group))
                ops.append(dist.P2POp(dist.isend, sv[c:d], dst, self.group))
            if self.rrows[src]:
                ops.append(dist.P2POp(dist.irecv, self.Blen[self.roff_r[src]:self.roff_r[src + 1]], src, self.group))
            if self.rnnz[src]:
                a, b = self.roff_n[src], self.roff_n[src + 1]
                ops.append(dist.P2POp(dist.irecv, self.Bcol[a:b], src, self.group))
                ops.append(dist.P2POp(dist.irecv, self.Bval[a:b], src, self.group))
        if ops:
            for r in dist.batch_isend_irecv(ops):
                r.wait()
        torch.cumsum(self.Blen, 0, out=self.Bptr[1:])
        return self.Bptr, self.Bcol, self.Bval

    def local_A(self) -> Block:
        """This rank's A block with columns renumbered to local B rows."""
        return Block(self.blk.r0, self.blk.r1, self.blk.ptr, self.acol_local, self.blk.val)


def spgemm_planned(plan: ShardPlan, multiply, gather: bool = False):
    """One row-sharded step with a planned exchange: exchange(B rows), local
    multiply (A's renumbered columns against the local B), optional gatherv."""
    Bptr, Bcol, Bval = plan.exchange()
    C = multiply(plan.local_A(), Bptr, Bcol, Bval, plan.M_global)
    g = gather_result(C, plan.blk, plan.group) if gather else None
    return C, g
