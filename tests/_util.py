"""Shared test helpers (test infrastructure)."""
from __future__ import annotations

import json
from pathlib import Path

import numpy as np

GOLDEN = Path(__file__).resolve().parent / "golden"


def load_golden(name: str):
    d = json.loads((GOLDEN / f"{name}.json").read_text())
    ptr = np.asarray(d["ptr"], np.int32)
    col = np.asarray(d["col"], np.int32)
    val = np.asarray([float.fromhex(x) for x in d["val_hex"]], np.float64)
    return d, ptr, col, val


PRODUCT_CASES = ["cage4_like", "tile_edges", "dense_row_col", "duplicates", "rect_AB", "empty_product"]
READ_CASES = ["mm_symmetric", "mm_skew", "mm_hermitian", "mm_pattern", "mm_integer", "mm_dups_comments"]


def csr_from_arrays(M, N, ptr, col, val):
    import mhspgemm
    return mhspgemm.CSR(M, N, ptr, col, val)


def random_csr(M, N, per_row, seed, lo=0.1, hi=1.0, sorted_unique=True, signed=False):
    rng = np.random.default_rng(seed)
    lens = rng.poisson(per_row, M)
    rows = np.repeat(np.arange(M), lens)
    cols = rng.integers(0, N, len(rows))
    key = np.unique(rows.astype(np.int64) * N + cols) if sorted_unique else rows.astype(np.int64) * N + cols
    r = key // N
    c = (key % N).astype(np.int32)
    ptr = np.zeros(M + 1, np.int64)
    np.cumsum(np.bincount(r, minlength=M), out=ptr[1:])
    v = rng.uniform(lo, hi, len(c))
    if signed:
        v *= rng.choice([-1.0, 1.0], len(c))
    return ptr.astype(np.int32), c, v


def bin_zoo(seed: int = 11):
    """A (rows of every kind) x B (K x N, N = 2M columns) such that rows land in
    every symbolic and numeric bin, including both global-memory fallbacks:
    empty, single product, banded (direct tables), scattered (hashed tables)
    of growing size, heavy work on a tiny pattern (duplicate A entries)."""
    rng = np.random.default_rng(seed)
    N = 2_000_000
    K = 3000
    # B rows: 0..499 tile [0, 32000) with 64 consecutive cols each, 500..999 "band" (64 consecutive
    # cols, 1000 apart), 1000..2998 "scatter" (50 random cols), row 2999 single entry
    Brows, Bcols = [], []
    for k in range(K):
        if k == K - 1:
            cs = np.array([12345])
        elif k < 500:                                # contiguous tiling of [0, 32000)
            cs = np.arange(64 * k, 64 * k + 64)
        elif k < 1000:
            off = 1000 * k % (N - 64)
            cs = np.arange(off, off + 64)
        else:
            cs = np.unique(rng.integers(0, N, 50))
        Brows.append(np.full(len(cs), k))
        Bcols.append(cs)
    Br = np.concatenate(Brows)
    Bc = np.concatenate(Bcols)
    Bkey = Br.astype(np.int64) * N + Bc
    order = np.argsort(Bkey, kind="stable")
    Br, Bc = Br[order], Bc[order]
    Bptr = np.zeros(K + 1, np.int64)
    np.cumsum(np.bincount(Br, minlength=K), out=Bptr[1:])
    Bv = rng.uniform(0.1, 1.0, len(Bc))

    arows = []  # list of lists of k (A entries, in order, duplicates allowed)
    arows.append([])                                 # empty
    arows.append([K - 1])                            # single product
    for i in range(20):                              # banded, small: direct, wave
        s = int(rng.integers(0, 990))
        arows.append(list(range(s, s + 8)))
    for i in range(10):                              # scattered small: hash, wave
        arows.append(sorted(rng.choice(np.arange(1000, K - 1), 2, replace=False).tolist()))
    for i in range(10):                              # scattered small-medium: hash, 16 KiB wave
        arows.append(sorted(rng.choice(np.arange(1000, K - 1), 4, replace=False).tolist()))
    for nb in (1, 3, 6, 9):                          # scattered rows of 50..450 products (tiny classes)
        for i in range(4):
            arows.append(sorted(rng.choice(np.arange(1000, K - 1), nb, replace=False).tolist()))
    for i in range(4):                               # > 512 products, 50 tiles: hash, wave
        arows.append([int(rng.integers(1000, K - 1))] * 12)
    for i in range(4):                               # > 512 products, ~300 tiles: hash, 256-thread block
        arows.append(sorted(rng.choice(np.arange(1000, K - 1), 6, replace=False).tolist() * 2))
    for i in range(4):                               # > 512 products, ~200 tiles: hash, 10 KiB wave
        arows.append(sorted(rng.choice(np.arange(1000, K - 1), 4, replace=False).tolist() * 3))
    for i in range(6):                               # scattered medium: hash, 256-thread block
        arows.append(sorted(rng.choice(np.arange(1000, K - 1), 20, replace=False).tolist()))
    for i in range(4):                               # scattered large: 1024-thread block
        arows.append(sorted(rng.choice(np.arange(1000, K - 1), 60, replace=False).tolist()))
    for i in range(2):                               # scattered huge: global memory
        arows.append(sorted(rng.choice(np.arange(1000, K - 1), 400, replace=False).tolist()))
    arows.append([5] * 3000)                         # heavy work, tiny pattern (duplicates)
    arows.append(list(range(0, 330)))                # 21120 contiguous columns, direct: global memory
    arows.append(sorted(rng.choice(np.arange(1000, K - 1), 120, replace=False).tolist()))  # wide: 1024 block
    arows.append(sorted(rng.choice(np.arange(0, 1000), 200, replace=False).tolist()))  # wide banded
    arows.append(list(range(0, 1000, 3)))            # direct, large span
    M = len(arows)
    Aptr = np.zeros(M + 1, np.int64)
    Aptr[1:] = np.cumsum([len(r) for r in arows])
    Acol = np.array([k for r in arows for k in r], np.int32)
    Av = rng.uniform(0.1, 1.0, len(Acol))
    return (M, K, Aptr.astype(np.int32), Acol, Av), (K, N, Bptr.astype(np.int32), Bc.astype(np.int32), Bv)


def run_zoo(seed: int = 5, N: int = 40_000):
    """B whose rows come in groups sharing one column pattern (runs of 1..7 rows,
    like the dofs of a FEM node), plus decoys: adjacent rows of equal length but
    different columns, and empty rows.  A rows walk consecutive B rows (runs, cut
    at 64-entry chunk edges and at the 3-row merge cap), skip rows (runs broken),
    repeat a row (k, k: not a run) and are long enough to reach the block and
    global kernels.  Exercises the same-pattern flag of the mask formation and the
    run walks of the symbolic and numeric phases."""
    rng = np.random.default_rng(seed)
    rows = []
    while len(rows) < 4000:
        kind = rng.integers(0, 10)
        if kind == 0:
            rows.append(np.zeros(0, np.int64))                       # empty row
            continue
        ln = int(rng.integers(1, 120))
        pat = np.unique(rng.integers(0, N, ln))
        if kind == 1:                                                # decoy: same length, new cols
            rows.append(pat)
            alt = np.unique(rng.integers(0, N, 4 * len(pat)))[:len(pat)]
            rows.append(np.sort(alt))
            continue
        rows.extend([pat] * int(rng.integers(1, 8)))                 # a run of 1..7 equal rows
    K = len(rows)
    Bptr = np.zeros(K + 1, np.int64)
    Bptr[1:] = np.cumsum([len(r) for r in rows])
    Bc = np.concatenate(rows).astype(np.int32)
    Bv = rng.uniform(0.1, 1.0, len(Bc))
    arows = []
    for i in range(600):
        kind = i % 6
        s = int(rng.integers(0, K - 400))
        if kind == 0:
            arows.append(list(range(s, s + int(rng.integers(1, 40)))))          # wave bins
        elif kind == 1:
            arows.append(list(range(s, s + int(rng.integers(60, 140)))))        # crosses chunk edges
        elif kind == 2:
            arows.append(sorted(set(rng.integers(s, s + 60, 30).tolist())))     # runs broken by gaps
        elif kind == 3:
            arows.append([s, s, s + 1, s + 1, s + 2])                           # repeats: not runs
        elif kind == 4:
            arows.append(list(range(s, s + 390)))                               # block / global kernels
        else:
            arows.append([])
    M = len(arows)
    Aptr = np.zeros(M + 1, np.int64)
    Aptr[1:] = np.cumsum([len(r) for r in arows])
    Acol = np.array([k for r in arows for k in r], np.int32)
    Av = rng.uniform(0.1, 1.0, len(Acol))
    return (M, K, Aptr.astype(np.int32), Acol, Av), (K, N, Bptr.astype(np.int32), Bc, Bv)


def group_zoo(seed: int = 3, K: int = 6000, N: int = 30_000):
    """A whose rows repeat column patterns (runs of 1..8 equal rows, so row groups of
    1..3 and runs cut by the group size and by the 96-row breaks), with small,
    medium and large patterns (grouped wave bins, the 16 KiB grouped bin, and
    groups too large for any grouped bin that run row by row); B random (K x N)
    with some same-pattern row runs of its own.  Values differ per row."""
    rng = np.random.default_rng(seed)
    arows = []
    while len(arows) < 700:
        size = int(rng.choice([2, 6, 20, 60, 200]))
        pat = np.unique(rng.integers(0, K, size))
        arows.extend([pat] * int(rng.integers(1, 9)))
        if rng.random() < 0.1:
            arows.append(np.zeros(0, np.int64))  # an empty row breaks a run
    M = len(arows)
    Aptr = np.zeros(M + 1, np.int64)
    Aptr[1:] = np.cumsum([len(r) for r in arows])
    Acol = np.concatenate(arows).astype(np.int32)
    Av = rng.uniform(0.1, 1.0, len(Acol))
    brows = []
    while len(brows) < K:
        pat = np.unique(rng.integers(0, N, int(rng.integers(1, 40))))
        brows.extend([pat] * int(rng.integers(1, 4)))
    brows = brows[:K]
    Bptr = np.zeros(K + 1, np.int64)
    Bptr[1:] = np.cumsum([len(r) for r in brows])
    Bc = np.concatenate(brows).astype(np.int32)
    Bv = rng.uniform(0.1, 1.0, len(Bc))
    return (M, K, Aptr.astype(np.int32), Acol, Av), (K, N, Bptr.astype(np.int32), Bc, Bv)


def tiny_zoo(seed: int = 7, K: int = 3000, N: int = 5000):
    """Rows for every tiny class (team of W lanes x K products per lane: flop <= 8, 32, 64
    with nA <= 8; <= 32, 64, 128 with nA <= 32; <= 256, 512 with nA <= 64), with colliding
    columns (B rows drawn from a narrow column window, repeated A entries) so segments of
    equal columns span lanes and slots, plus rows just past the limits (flop 513+, nA
    past the lane count with empty B rows)."""
    rng = np.random.default_rng(seed)
    brows = []
    for k in range(K):
        kind = k % 5
        if kind == 0:
            brows.append(np.zeros(0, np.int64))                                     # empty B row
        elif kind == 1:
            brows.append(np.unique(rng.integers(0, 200, int(rng.integers(1, 4)))))  # narrow: collisions
        else:
            brows.append(np.unique(rng.integers(0, N, int(rng.integers(1, 9)))))
    Bptr = np.zeros(K + 1, np.int64)
    Bptr[1:] = np.cumsum([len(r) for r in brows])
    Bc = np.concatenate(brows).astype(np.int32)
    Bv = rng.uniform(0.1, 1.0, len(Bc))
    blen = np.diff(Bptr)
    nonempty = np.nonzero(blen)[0]
    empty = np.nonzero(blen == 0)[0]
    arows = []
    for target, amax in ((1, 8), (4, 8), (8, 8), (16, 8), (30, 8), (32, 8), (60, 8), (64, 8), (20, 32), (32, 32),
                         (50, 32), (64, 32), (100, 32), (128, 32),
                         (129, 32), (200, 64), (256, 64), (300, 64), (512, 64), (513, 64), (700, 64)):
        for _ in range(30):
            ks, f = [], 0
            for _try in range(600):
                if f >= target or len(ks) >= amax:
                    break
                k = int(rng.choice(nonempty))
                if f + blen[k] > target:
                    continue
                ks.append(k)
                f += int(blen[k])
                if rng.random() < 0.2 and f + blen[k] <= target and len(ks) < amax:
                    ks.append(k)  # repeated A entry: every product collides
                    f += int(blen[k])
            arows.append(sorted(ks))
    for na in (34, 66):  # many A entries, few products: past a class's lane count
        for _ in range(15):
            arows.append(sorted(rng.choice(empty, na, replace=False).tolist() + [int(rng.choice(nonempty))]))
    arows.append([])
    M = len(arows)
    Aptr = np.zeros(M + 1, np.int64)
    Aptr[1:] = np.cumsum([len(r) for r in arows])
    Acol = np.array([k for r in arows for k in r], np.int32)
    Av = rng.uniform(0.1, 1.0, len(Acol))
    return (M, K, Aptr.astype(np.int32), Acol, Av), (K, N, Bptr.astype(np.int32), Bc, Bv)


def near_zoo(seed: int = 4):
    """A x B for near row groups (GRP_NEAR): B a 27-point x 3-dof FEM grid, A its pattern
    with 5 % of the off-diagonal entries dropped per row (dof triples whose A rows differ
    by a few entries but whose C rows mostly coincide), and some rows made awkward: a far
    column appended (unsorted, and the row's C pattern no longer matches its triple's), an
    entry repeated (a duplicate column, summed), the row reversed (unsorted A)."""
    from mhspgemm import synth
    B = synth.fem_grid(12, 10, 8, seed=seed)
    rng = np.random.default_rng(seed)
    cols, vals, lens = [], [], []
    for i in range(B.M):
        c = B.col[B.ptr[i]:B.ptr[i + 1]].copy()
        v = rng.uniform(0.1, 1.0, len(c))
        keep = (c == i) | (rng.random(len(c)) >= 0.05)
        c, v = c[keep], v[keep]
        u = rng.random()
        if u < 0.04:
            c = np.append(c, rng.integers(0, B.M))
            v = np.append(v, 0.5)
        elif u < 0.07:
            j = int(rng.integers(0, len(c)))
            c = np.insert(c, j, c[j])
            v = np.insert(v, j, 0.25)
        elif u < 0.10:
            c, v = c[::-1].copy(), v[::-1].copy()
        cols.append(c)
        vals.append(v)
        lens.append(len(c))
    ptr = np.zeros(B.M + 1, np.int64)
    ptr[1:] = np.cumsum(lens)
    A = (B.M, B.M, ptr.astype(np.int32), np.concatenate(cols).astype(np.int32), np.concatenate(vals))
    return A, (B.M, B.N, B.ptr, B.col, B.val)
