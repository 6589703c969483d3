"""Deterministic synthetic stand-ins for the BASELINE.json matrices.

The SuiteSparse files of 16matrix.txt (reference process.sh:3-23 reads
../matrix/<name>/<name>.mtx) cannot be downloaded here.  When they are present,
``load_or_synth`` reads them from $MHS_MATRIX_DIR/<name>/<name>.mtx; otherwise
it builds a synthetic matrix with the same size and structural character.
All values are U(0.1, 1.0) (positive: no cancellation, so structural nnz equals
numerical nnz and any checker agrees on the pattern).

  S0 cage4-like   n=9, nnz=49: diagonal + 40 distinct off-diagonals
  S1 cant-like    FEM cantilever: 9 x 9 x 257 node grid, 27-point node stencil,
                  3 dof per node -> n = 62,451, ~69 nnz/row, nnz(A^2) ~281/row
                  (the real cant: 62,451 rows, ~64 nnz/row, nnz(C) ~279/row)
  S2 webbase-like n=1,000,005, power-law row lengths (discrete Pareto a=2.28, hub
                  rows to the 4,700 cap), local / site-navigation / Zipf-popular links,
                  popular pages = long rows (web_graph; calibrated in round 5)
  S3 sweep        mac_econ_fwd500-, scircuit-, cop20k_A-like (3-D geometric, round 5)
  S4 cage15-like  n=5,154,859, ~19 nnz/row, near-diagonal + 10% long range
"""
from __future__ import annotations

import os
from pathlib import Path

import numpy as np

from .core import CSR, readMtxFile


def _csr_from_coo(n_rows, n_cols, r, c, rng, values=None) -> CSR:
    r = np.asarray(r, np.int64)
    c = np.asarray(c, np.int64)
    key = np.unique(r * n_cols + c)  # sorted, deduplicated
    rows = key // n_cols
    cols = (key - rows * n_cols).astype(np.int32)
    ptr = np.zeros(n_rows + 1, np.int64)
    np.cumsum(np.bincount(rows, minlength=n_rows), out=ptr[1:])
    val = rng.uniform(0.1, 1.0, size=len(cols)) if values is None else values(len(cols))
    return CSR(n_rows, n_cols, ptr.astype(np.int32), cols, val.astype(np.float64))


def cage4_like(seed: int = 1) -> CSR:
    rng = np.random.default_rng(seed)
    n = 9
    off = [(i, j) for i in range(n) for j in range(n) if i != j]
    pick = rng.choice(len(off), size=40, replace=False)
    r = [i for i in range(n)] + [off[k][0] for k in pick]
    c = [i for i in range(n)] + [off[k][1] for k in pick]
    return _csr_from_coo(n, n, r, c, rng)


def fem_grid(nx: int, ny: int, nz: int, dof: int = 3, seed: int = 2) -> CSR:
    """27-point node stencil on an nx*ny*nz grid, `dof` unknowns per node (node
    index x + nx*(y + ny*z), unknown index dof*node + d)."""
    rng = np.random.default_rng(seed)
    x, y, z = np.meshgrid(np.arange(nx), np.arange(ny), np.arange(nz), indexing="ij")
    x, y, z = x.ravel(), y.ravel(), z.ravel()
    node = x + nx * (y + ny * z)
    rs, cs = [], []
    for dx in (-1, 0, 1):
        for dy in (-1, 0, 1):
            for dz in (-1, 0, 1):
                xx, yy, zz = x + dx, y + dy, z + dz
                ok = (xx >= 0) & (xx < nx) & (yy >= 0) & (yy < ny) & (zz >= 0) & (zz < nz)
                a = node[ok]
                b = (xx + nx * (yy + ny * zz))[ok]
                for d in range(dof):
                    for e in range(dof):
                        rs.append(dof * a + d)
                        cs.append(dof * b + e)
    n = nx * ny * nz * dof
    return _csr_from_coo(n, n, np.concatenate(rs), np.concatenate(cs), rng)


def cant_like(seed: int = 2) -> CSR:
    return fem_grid(9, 9, 257, 3, seed)


def powerlaw(n: int, alpha: float = 2.1, cap: int = 4700, local_frac: float = 0.7,
             local_width: int = 1024, zipf_s: float = 1.2, seed: int = 3) -> CSR:
    """webbase-like: Pareto row lengths, columns local or Zipf-popular."""
    rng = np.random.default_rng(seed)
    u = rng.random(n)
    lens = np.floor((1.0 - u) ** (-1.0 / (alpha - 1.0))).astype(np.int64)
    lens = np.clip(lens, 1, cap)
    total = int(lens.sum())
    rows = np.repeat(np.arange(n, dtype=np.int64), lens)
    local = rng.random(total) < local_frac
    cols = np.empty(total, np.int64)
    nl = int(local.sum())
    cols[local] = rows[local] + rng.integers(-local_width, local_width + 1, size=nl)
    # Zipf popularity over a random permutation of the columns
    nz = total - nl
    ranks = rng.zipf(zipf_s, size=nz) - 1
    ranks = np.minimum(ranks, n - 1)
    perm = rng.permutation(n)
    cols[~local] = perm[ranks]
    cols = np.clip(cols, 0, n - 1)
    return _csr_from_coo(n, n, rows, cols, rng)


def web_graph(n: int, alpha: float = 2.277, cap: int = 4700, nbig: int = 10, local_frac: float = 0.361,
              local_width: int = 128, nav_frac: float = 0.252, site: int = 32, zipf_s: float = 1.194,
              hubk: int = 5, hubskip: int = 800, seed: int = 3) -> CSR:
    """webbase-like (round 5, calibrated to the SuiteSparse statistics of webbase-1M):
    Pareto row lengths (the nbig longest raised towards the 4,700 cap: hub pages), and per entry a
    local link (within +-local_width of the page; hub rows over 4x their length), a site
    navigation link (the first pages of the page's site of `site` pages, Zipf-weighted: pages of
    one site share them -- the overlap that puts nnz(C) below flop) or a Zipf-popular page; the
    `hubk` most popular pages are long rows (ranks hubskip.. of the length order), which is where
    the products of a web graph's A*A come from."""
    rng = np.random.default_rng(seed)
    u = rng.random(n)
    lens = np.clip(np.floor((1.0 - u) ** (-1.0 / (alpha - 1.0))).astype(np.int64), 1, cap)
    big = np.argsort(-lens, kind="stable")[:nbig]
    lens[big] = np.maximum(lens[big], np.linspace(cap, cap // 3, nbig).astype(np.int64))
    total = int(lens.sum())
    rows = np.repeat(np.arange(n, dtype=np.int64), lens)
    rl = np.repeat(lens, lens)
    kind = rng.random(total)
    hub = rl > 1000
    local = (kind < local_frac) | hub
    nav = ~hub & (kind >= local_frac) & (kind < local_frac + nav_frac)
    far = ~hub & (kind >= local_frac + nav_frac)
    cols = np.empty(total, np.int64)
    w = np.where(rl[local] > 1000, 4 * rl[local], np.maximum(local_width, rl[local]))
    cols[local] = rows[local] + (rng.random(int(local.sum())) * (2 * w + 1)).astype(np.int64) - w
    cols[nav] = (rows[nav] // site) * site + np.minimum(rng.zipf(2.0, size=int(nav.sum())) - 1, site - 1)
    ranks = np.minimum(rng.zipf(zipf_s, size=int(far.sum())) - 1, n - 1)
    perm = rng.permutation(n)
    pos = np.empty(n, np.int64)
    pos[perm] = np.arange(n)
    for r, row in enumerate(np.argsort(-lens, kind="stable")[hubskip:hubskip + hubk]):
        j = pos[row]
        perm[r], perm[j] = perm[j], perm[r]
        pos[perm[r]], pos[perm[j]] = r, j
    cols[far] = perm[ranks]
    cols = np.clip(cols, 0, n - 1)
    return _csr_from_coo(n, n, rows, cols, rng)


def webbase_like(seed: int = 3) -> CSR:
    return web_graph(1_000_005, seed=seed)


def banded_random(n: int, per_row: float, width: int, far_frac: float = 0.0, seed: int = 7,
                  diag: bool = True) -> CSR:
    """Rows with ~per_row entries within +-width of the diagonal, a fraction
    far_frac of them uniform over all columns."""
    rng = np.random.default_rng(seed)
    lens = rng.poisson(per_row, size=n).astype(np.int64)
    lens = np.maximum(lens, 1)
    rows = np.repeat(np.arange(n, dtype=np.int64), lens)
    total = len(rows)
    cols = rows + rng.integers(-width, width + 1, size=total)
    far = rng.random(total) < far_frac
    cols[far] = rng.integers(0, n, size=int(far.sum()))
    cols = np.clip(cols, 0, n - 1)
    if diag:
        rows = np.concatenate([rows, np.arange(n)])
        cols = np.concatenate([cols, np.arange(n)])
    return _csr_from_coo(n, n, rows, cols, rng)


def mac_econ_like(seed: int = 4, cluster: int = 600, far_frac: float = 0.10) -> CSR:
    """Block-diagonal clusters of `cluster` rows at ~6.2 nnz/row (diagonal included) plus sparse
    coupling (`far_frac` of the entries uniform over the columns).  Round 6: recalibrated to the
    SuiteSparse statistics (TARGETS) -- clusters of 600 instead of 50 rows, 10 % coupling: the
    round-1..5 stand-in's clusters repeated columns within a C row, nnz(C) 73 % of the real one."""
    rng = np.random.default_rng(seed)
    n = 206_500
    lens = np.maximum(rng.poisson(5.2, size=n), 1).astype(np.int64)
    rows = np.repeat(np.arange(n, dtype=np.int64), lens)
    blk = rows // cluster
    cols = blk * cluster + rng.integers(0, cluster, size=len(rows))
    far = rng.random(len(rows)) < far_frac
    cols[far] = rng.integers(0, n, size=int(far.sum()))
    cols = np.clip(cols, 0, n - 1)
    rows = np.concatenate([rows, np.arange(n)])
    cols = np.concatenate([cols, np.arange(n)])
    return _csr_from_coo(n, n, rows, cols, rng)


def sym_banded(n: int, per_side: float, width: int, far_frac: float, disp: float = 0.0, seed: int = 7) -> CSR:
    """Structurally symmetric rows: `per_side` entries per row drawn within +-width of the diagonal
    (a `far_frac` share uniform over the columns), mirrored (pattern of X + X^T), diagonal included.
    Row degrees are Poisson, or gamma-Poisson (negative binomial) with shape `disp` when > 0: for a
    symmetric pattern flop / row = E[deg^2], so the degree spread sets the products."""
    rng = np.random.default_rng(seed)
    lam = rng.gamma(disp, per_side / disp, size=n) if disp > 0 else per_side
    lens = rng.poisson(lam, size=n).astype(np.int64)
    rows = np.repeat(np.arange(n, dtype=np.int64), lens)
    cols = rows + rng.integers(-width, width + 1, size=len(rows))
    far = rng.random(len(rows)) < far_frac
    cols[far] = rng.integers(0, n, size=int(far.sum()))
    cols = np.clip(cols, 0, n - 1)
    d = np.arange(n, dtype=np.int64)
    return _csr_from_coo(n, n, np.concatenate([rows, cols, d]), np.concatenate([cols, rows, d]), rng)


def scircuit_like(seed: int = 5) -> CSR:
    """Circuit: a structurally symmetric near-diagonal pattern of widely spread degrees (~5.6
    entries a row) plus 10 hub nets (rows / columns of ~350 entries).  Round 6: recalibrated to the
    SuiteSparse statistics (TARGETS; round 1..5: an unsymmetric band plus 20 hubs, flop 79 % and
    nnz(C) 118 % of the real ones)."""
    rng = np.random.default_rng(seed + 100)
    n = 170_998
    base = sym_banded(n, 2.65, 16, 0.02, disp=0.5, seed=seed)
    hubs = rng.choice(n, size=10, replace=False)
    r = [np.repeat(np.arange(n), np.diff(base.ptr))]
    c = [base.col.astype(np.int64)]
    for h in hubs:
        others = rng.choice(n, size=350, replace=False)
        r += [np.full(350, h), others]
        c += [others, np.full(350, h)]
    return _csr_from_coo(n, n, np.concatenate(r), np.concatenate(c), rng)


def cop20k_like(seed: int = 6, density: float = 5.0, degree: float = 14.5, far: float = 0.75) -> CSR:
    """cop20k_A-like (round 5, calibrated to SURVEY §8's statistics): a random geometric graph of
    121,192 points in the unit cube whose density varies by a factor 1 + `density` across it
    (degrees 1..~70: the size-biased degree sets flop), linked within the radius of mean degree
    `degree`, plus a random long link for a fraction `far` of the points (C rows grow by a
    neighbour's row each), diagonal included; rows numbered along z-slabs of a 48^3 cell grid
    (banded columns).  The round-1..4 2-D grid stand-in had 65 % of the flop and 44 % of nnz(C)."""
    from scipy.spatial import cKDTree
    rng = np.random.default_rng(seed)
    n = 121_192
    pts, need = [], n
    while need > 0:
        p = rng.random((need * 3, 3))
        f = (1 + density * np.sin(3.1 * p[:, 0]) ** 2 * np.cos(2.3 * p[:, 2]) ** 2) / (1 + density)
        p = p[rng.random(len(p)) < f][:need]
        pts.append(p)
        need -= len(p)
    P = np.concatenate(pts)[:n]
    r = (degree / (n * 4.0 / 3.0 * np.pi)) ** (1.0 / 3.0)
    pr = cKDTree(P).query_pairs(r, output_type="ndarray")
    cell = np.floor(P * 48).astype(np.int64)
    rank = np.empty(n, np.int64)
    rank[np.lexsort((cell[:, 0], cell[:, 1], cell[:, 2]))] = np.arange(n)
    a, b = rank[pr[:, 0]], rank[pr[:, 1]]
    fa = np.nonzero(rng.random(n) < far)[0]
    fb = rng.integers(0, n, len(fa))
    rs = np.concatenate([a, b, fa, fb, np.arange(n)])
    cs = np.concatenate([b, a, fb, fa, np.arange(n)])
    return _csr_from_coo(n, n, rs, cs, rng)


def cop20k_grid2d(seed: int = 6) -> CSR:
    """The round-1..4 cop20k_A stand-in: a random geometric graph on a 2-D grid, ~21.7 nnz/row."""
    rng = np.random.default_rng(seed)
    n = 121_192
    side = int(np.ceil(np.sqrt(n)))
    pos = rng.permutation(side * side)[:n]
    px, py = pos % side, pos // side
    order = np.lexsort((px, py))  # rows numbered along the grid
    px, py = px[order], py[order]
    cell = {}
    grid = np.full((side, side), -1, np.int64)
    grid[py, px] = np.arange(n)
    rs, cs = [], []
    for dx in range(-2, 3):
        for dy in range(-2, 3):
            if dx * dx + dy * dy > 5:
                continue
            xx, yy = px + dx, py + dy
            ok = (xx >= 0) & (xx < side) & (yy >= 0) & (yy < side)
            nb = np.full(n, -1, np.int64)
            nb[ok] = grid[yy[ok], xx[ok]]
            good = nb >= 0
            rs.append(np.arange(n)[good])
            cs.append(nb[good])
    del cell
    return _csr_from_coo(n, n, np.concatenate(rs), np.concatenate(cs), rng)


def cage15_like(seed: int = 7) -> CSR:
    """cage15 (DNA electrophoresis, structurally symmetric): ~19.3 entries a row within +-48 of
    the diagonal, 5.8 % long-range, degrees gamma-Poisson spread.  Round 6: recalibrated to the
    SuiteSparse statistics (TARGETS: flop 2.08e9, nnz(C) 9.29e8 -- 2.24 products per C entry).
    The round-1..5 stand-in (cage15_banded: an unsymmetric +-300 band, 10 % far) had 1.19 products
    per C entry: nnz(C) 168 % and flop 89 % of the real matrix."""
    return sym_banded(5_154_859, 10.25, 48, 0.058, disp=3.5, seed=seed)


def cage15_banded(seed: int = 7) -> CSR:
    """The round-1..5 cage15 stand-in (kept for comparison with earlier records)."""
    return banded_random(5_154_859, 18.2, 300, far_frac=0.10, seed=seed)


# ---- headline robustness variants ---------------------------

def cant_s1(seed: int = 2) -> CSR:
    """SURVEY §8(d) S1 exactly as specified: n = 62,451, every row 64 entries as 4
    runs of 16 consecutive columns placed at random within +-1,500 of the diagonal,
    then symmetrised (pattern of A + A^T; the mirrored entry takes the row's value
    where both exist).  No dof structure: rows do not repeat their neighbours'
    patterns, so the row-group path does not fire."""
    rng = np.random.default_rng(seed)
    n = 62_451
    starts = np.arange(n)[:, None] + rng.integers(-1500, 1500 - 16 + 1, size=(n, 4))
    starts = np.clip(starts, 0, n - 16)
    cols = (starts[:, :, None] + np.arange(16)[None, None, :]).reshape(n, 64)
    rows = np.repeat(np.arange(n, dtype=np.int64), 64)
    cols = cols.reshape(-1).astype(np.int64)
    r = np.concatenate([rows, cols])
    c = np.concatenate([cols, rows])
    return _csr_from_coo(n, n, r, c, rng)


def cant_perturbed(seed: int = 2, drop: float = 0.03) -> CSR:
    """cant-like (27-point x 3-dof FEM grid) with `drop` of its off-diagonal entries
    removed at random (not symmetrically): dof runs and row groups break where an
    entry is missing, as boundary conditions and pruned entries do in the real cant."""
    A = cant_like(seed)
    rng = np.random.default_rng(seed + 1000)
    rows = np.repeat(np.arange(A.M, dtype=np.int64), np.diff(A.ptr))
    keep = (rows == A.col) | (rng.random(A.nnz) >= drop)
    ptr = np.zeros(A.M + 1, np.int64)
    np.cumsum(np.bincount(rows[keep], minlength=A.M), out=ptr[1:])
    return CSR(A.M, A.N, ptr.astype(np.int32), A.col[keep], A.val[keep])


# ---- stand-ins for the rest of 16matrix.txt (reference 16matrix.txt:1-16) --------

def fem_stencil(dims, dof: int, stencil: str = "27", seed: int = 2) -> CSR:
    """Node stencil on a 2-D or 3-D grid (`stencil` "27": every neighbour incl.
    diagonals -- 9 in 2-D; "7": face neighbours -- 5 in 2-D), `dof` unknowns per node."""
    if len(dims) == 2:
        dims = (dims[0], dims[1], 1)
    nx, ny, nz = dims
    if stencil == "27":
        offs = [(dx, dy, dz) for dx in (-1, 0, 1) for dy in (-1, 0, 1) for dz in (-1, 0, 1)]
    else:
        offs = [(0, 0, 0), (1, 0, 0), (-1, 0, 0), (0, 1, 0), (0, -1, 0), (0, 0, 1), (0, 0, -1)]
    offs = [o for o in offs if nz > 1 or o[2] == 0]
    rng = np.random.default_rng(seed)
    x, y, z = np.meshgrid(np.arange(nx), np.arange(ny), np.arange(nz), indexing="ij")
    x, y, z = x.ravel(), y.ravel(), z.ravel()
    node = x + nx * (y + ny * z)
    rs, cs = [], []
    for dx, dy, dz in offs:
        xx, yy, zz = x + dx, y + dy, z + dz
        ok = (xx >= 0) & (xx < nx) & (yy >= 0) & (yy < ny) & (zz >= 0) & (zz < nz)
        a, b = node[ok], (xx + nx * (yy + ny * zz))[ok]
        for d in range(dof):
            for e in range(dof):
                rs.append(dof * a + d)
                cs.append(dof * b + e)
    n = nx * ny * nz * dof
    return _csr_from_coo(n, n, np.concatenate(rs), np.concatenate(cs), rng)


def _tiled_order(side_x: int, side_y: int, tile: int = 32) -> np.ndarray:
    """Node numbering of a side_x x side_y grid by tile x tile blocks (row-major
    blocks, row-major inside): graph neighbours stay within a few thousand ids."""
    x, y = np.meshgrid(np.arange(side_x), np.arange(side_y), indexing="xy")
    x, y = x.ravel(), y.ravel()
    tx, ty = x // tile, y // tile
    ntx = (side_x + tile - 1) // tile
    key = ((ty * ntx + tx) * tile + (y % tile)) * tile + (x % tile)
    order = np.empty(len(key), np.int64)
    order[np.argsort(key, kind="stable")] = np.arange(len(key))
    return order.reshape(side_y, side_x)


def road_like(n: int = 23_947_347, p: float = 0.6, seed: int = 8) -> CSR:
    """GAP-road-like: a planar road network of ~2.4 entries per row, symmetric, no
    diagonal: the edges of a grid (right and down neighbours, each kept with
    probability p: mean degree 4p) on tiled node ids."""
    rng = np.random.default_rng(seed)
    side = int(np.ceil(np.sqrt(n)))
    ids = _tiled_order(side, side)
    rs, cs = [], []
    for dx, dy in ((1, 0), (0, 1)):
        a = ids[: side - dy, : side - dx].ravel()
        b = ids[dy:, dx:].ravel()
        keep = (rng.random(len(a)) < p) & (a < n) & (b < n)
        rs += [a[keep], b[keep]]
        cs += [b[keep], a[keep]]
    return _csr_from_coo(n, n, np.concatenate(rs), np.concatenate(cs), rng)


def delaunay_like(side: int = 4096, seed: int = 9) -> CSR:
    """delaunay_n24-like (2^24 points, ~6 entries per row, no diagonal): a grid
    triangulated with a random diagonal per cell (mean degree 6, varying), tiled ids."""
    rng = np.random.default_rng(seed)
    n = side * side
    ids = _tiled_order(side, side)
    rs, cs = [], []
    for dx, dy in ((1, 0), (0, 1)):
        a, b = ids[: side - dy, : side - dx].ravel(), ids[dy:, dx:].ravel()
        rs += [a, b]
        cs += [b, a]
    flip = rng.random((side - 1, side - 1)) < 0.5
    a = np.where(flip, ids[:-1, :-1], ids[:-1, 1:]).ravel()   # (x,y)-(x+1,y+1) or (x+1,y)-(x,y+1)
    b = np.where(flip, ids[1:, 1:], ids[1:, :-1]).ravel()
    rs += [a, b]
    cs += [b, a]
    return _csr_from_coo(n, n, np.concatenate(rs), np.concatenate(cs), rng)


def wb_edu_like(seed: int = 10) -> CSR:
    """wb-edu-like: 9,845,725 rows of a power-law web crawl, ~5.8 entries per row,
    mostly site-local links plus Zipf-popular hubs."""
    return powerlaw(9_845_725, alpha=2.12, cap=4700, local_frac=0.8, local_width=2048, zipf_s=1.2, seed=seed)


def offshore_like(seed: int = 11) -> CSR:
    """offshore-like: 3-D 7-point stencil x 2 dof (~14/row) on 64 x 64 x 32 nodes plus
    a few random local couplings (~16/row): n = 262,144 (real 259,789)."""
    A = fem_stencil((64, 64, 32), 2, "7", seed=seed)
    rng = np.random.default_rng(seed)
    rows = np.repeat(np.arange(A.M, dtype=np.int64), np.diff(A.ptr))
    extra = rng.integers(0, A.M, A.M)
    er = (extra + rng.integers(-3000, 3001, A.M)) % A.M
    r = np.concatenate([rows, extra, er])
    c = np.concatenate([A.col.astype(np.int64), er, extra])
    return _csr_from_coo(A.M, A.N, r, c, rng)


SYNTH = {
    "cage4": cage4_like,
    "cant": cant_like,
    "webbase-1M": webbase_like,
    "mac_econ_fwd500": mac_econ_like,
    "scircuit": scircuit_like,
    "cop20k_A": cop20k_like,
    "cage15": cage15_like,
    "cage15-r5": cage15_banded,
    # cage15-like without its long-range entries (the near band's share of the traffic)
    "cage15-near": lambda: sym_banded(5_154_859, 10.25, 48, 0.0, disp=3.5, seed=7),
    # headline robustness variants
    "cant-s1": cant_s1,
    "cant-perturbed": cant_perturbed,
    # the rest of 16matrix.txt
    "pdb1HYS": lambda: fem_stencil((11, 11, 75), 4, "27", seed=12),     # n 36,300 (real 36,417), ~100/row
    "pwtk": lambda: fem_stencil((31, 31, 113), 2, "27", seed=13),       # n 217,186 (real 217,918), ~50/row
    "cage12": lambda: banded_random(130_228, 14.6, 300, far_frac=0.10, seed=14),  # ~15.6/row
    "hood": lambda: fem_stencil((10, 10, 1103), 2, "27", seed=15),      # n 220,600 (real 220,542), ~45/row
    "rma10": lambda: fem_stencil((88, 88), 6, "27", seed=16),           # 2-D, n 46,464 (real 46,835), ~52/row
    "shipsec1": lambda: fem_stencil((40, 40, 44), 2, "27", seed=17),    # n 140,800 (real 140,874), ~50/row
    "offshore": offshore_like,
    "wb-edu": wb_edu_like,
    "GAP-road": road_like,
    "delaunay_n24": delaunay_like,
}

# SuiteSparse statistics of the BASELINE.json config matrices (external metadata,
# ~ values; nnz(A) of symmetric files expanded) beside what the stand-ins achieve (this module,
# counted here on the CPU: tests/test_host.py::test_standin_stats re-counts the cheap ones)
TARGETS = {
    "cant": dict(M=62_451, nnzA=4.0e6, flop=2.70e8, nnzC=1.74e7),
    "webbase-1M": dict(M=1_000_005, nnzA=3.1e6, flop=6.95e7, nnzC=5.1e7, max_row=4700),
    "mac_econ_fwd500": dict(M=206_500, nnzA=1.27e6, flop=7.6e6, nnzC=6.7e6),
    "scircuit": dict(M=170_998, nnzA=0.96e6, flop=8.7e6, nnzC=5.2e6),
    "cop20k_A": dict(M=121_192, nnzA=2.62e6, flop=8.0e7, nnzC=1.87e7, max_row=81),
    "cage15": dict(M=5_154_859, nnzA=9.92e7, flop=2.08e9, nnzC=9.29e8),
}
ACHIEVED = {
    "cant": dict(M=62_451, nnzA=4_325_625, flop=313_454_421, nnzC=17_508_231),
    "webbase-1M": dict(M=1_000_005, nnzA=3_262_448, flop=60_394_619, nnzC=57_825_754, max_row=4454),
    "mac_econ_fwd500": dict(M=206_500, nnzA=1_277_478, flop=7_902_501, nnzC=6_709_169, max_row=19),
    "scircuit": dict(M=170_998, nnzA=941_226, flop=8_359_752, nnzC=5_333_138, max_row=365),
    "cop20k_A": dict(M=121_192, nnzA=2_668_988, flop=75_941_018, nnzC=18_902_088, max_row=73),
    "cage15": dict(M=5_154_859, nnzA=99_497_451, flop=2_097_991_939, nnzC=934_229_145, max_row=60),
}
# how close each stand-in is held to TARGETS (relative, every listed statistic; test_standin_stats):
# cant-like is the 27-point x 3-dof FEM grid of the real cant's size (its stencil sets the counts)
CALIBRATED_TOL = {"cant": 0.17, "webbase-1M": 0.14, "mac_econ_fwd500": 0.05, "scircuit": 0.05,
                  "cop20k_A": 0.10, "cage15": 0.05}

# reference 16matrix.txt, in its order (process.sh:21-37 walks it)
MATRIX16 = ["pdb1HYS", "pwtk", "webbase-1M", "cage12", "cant", "hood", "rma10", "scircuit", "shipsec1",
            "cop20k_A", "mac_econ_fwd500", "offshore", "wb-edu", "cage15", "GAP-road", "delaunay_n24"]


def matrix_path(name: str) -> Path | None:
    root = os.environ.get("MHS_MATRIX_DIR")
    if not root:
        return None
    p = Path(root) / name / f"{name}.mtx"
    return p if p.exists() else None


def _cached(name: str) -> CSR:
    """SYNTH[name](), memoised as .npz under $MHS_SYNTH_CACHE when that is set
    (the big stand-ins take tens of seconds to generate; several processes of one
    GPU job then build them once)."""
    root = os.environ.get("MHS_SYNTH_CACHE")
    if not root:
        return SYNTH[name]()
    f = Path(root) / f"{name}.npz"
    if f.exists():
        d = np.load(f)
        return CSR(int(d["M"]), int(d["N"]), d["ptr"], d["col"], d["val"])
    A = SYNTH[name]()
    f.parent.mkdir(parents=True, exist_ok=True)
    tmp = f.with_suffix(f".{os.getpid()}.npz")
    np.savez(tmp, M=A.M, N=A.N, ptr=A.ptr, col=A.col, val=A.val)
    os.replace(tmp, f)
    return A


def load_or_synth(name: str) -> tuple[CSR, str]:
    """The real matrix if $MHS_MATRIX_DIR/<name>/<name>.mtx exists, else the
    synthetic stand-in.  Returns (A, source description)."""
    p = matrix_path(name)
    if p is not None:
        A = CSR()
        if readMtxFile(A, str(p)) == 0:
            return A, f"file:{p}"
    if name not in SYNTH:
        raise KeyError(f"no synthetic stand-in for {name!r}")
    return _cached(name), f"synthetic:{name}-like"


# ---- one host copy for several ranks (bench.py --gpus N) --------------------------

def shared_dir(name: str) -> Path:
    root = os.environ.get("MHS_SYNTH_CACHE") or f"/tmp/mhs_synth_{os.getuid()}"
    return Path(root) / f"{name}.csr"


def build_shared(name: str) -> str:
    """Write `name`'s matrix (the file, else the stand-in) as ptr/col/val .npy files
    under shared_dir(name) unless they exist; returns the source description.  One
    process per node calls this; the others then `open_shared` (memory-mapped: a rank
    touches only the pages of its row block)."""
    d = shared_dir(name)
    src = d / "source.txt"
    if src.exists():
        return src.read_text()
    A, source = load_or_synth(name)
    tmp = d.with_name(f"{d.name}.{os.getpid()}.tmp")
    tmp.mkdir(parents=True, exist_ok=True)
    np.save(tmp / "ptr.npy", A.ptr)
    np.save(tmp / "col.npy", A.col)
    np.save(tmp / "val.npy", A.val)
    (tmp / "shape.txt").write_text(f"{A.M} {A.N}")
    (tmp / "source.txt").write_text(source)
    try:
        os.replace(tmp, d)
    except OSError:  # another process got there first
        import shutil
        shutil.rmtree(tmp, ignore_errors=True)
    return (d / "source.txt").read_text()


def open_shared(name: str):
    """(M, N, ptr, col, val, source) of build_shared's files, col/val memory-mapped."""
    d = shared_dir(name)
    M, N = (int(x) for x in (d / "shape.txt").read_text().split())
    ptr = np.load(d / "ptr.npy")
    col = np.load(d / "col.npy", mmap_mode="r")
    val = np.load(d / "val.npy", mmap_mode="r")
    return M, N, ptr, col, val, (d / "source.txt").read_text()
