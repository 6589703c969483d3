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
  S2 webbase-like n=1,000,005, power-law row lengths (discrete Pareto a=2.1, cap
                  4,700), 70% local / 30% Zipf-popular columns: long C rows
  S3 sweep        mac_econ_fwd500-, scircuit-, cop20k_A-like
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


def webbase_like(seed: int = 3) -> CSR:
    return powerlaw(1_000_005, seed=seed)


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


def mac_econ_like(seed: int = 4) -> CSR:
    """Block-diagonal clusters of ~50 rows at ~6.2 nnz/row plus sparse coupling."""
    rng = np.random.default_rng(seed)
    n = 206_500
    lens = np.maximum(rng.poisson(5.2, size=n), 1).astype(np.int64)
    rows = np.repeat(np.arange(n, dtype=np.int64), lens)
    blk = rows // 50
    cols = blk * 50 + rng.integers(0, 50, size=len(rows))
    far = rng.random(len(rows)) < 0.05
    cols[far] = rng.integers(0, n, size=int(far.sum()))
    cols = np.clip(cols, 0, n - 1)
    rows = np.concatenate([rows, np.arange(n)])
    cols = np.concatenate([cols, np.arange(n)])
    return _csr_from_coo(n, n, rows, cols, rng)


def scircuit_like(seed: int = 5) -> CSR:
    """Circuit: ~5.6 nnz/row near-diagonal plus 20 dense-ish rows/cols (~350 nnz)."""
    rng = np.random.default_rng(seed)
    n = 170_998
    base = banded_random(n, 4.0, 200, far_frac=0.1, seed=seed)
    hubs = rng.choice(n, size=20, replace=False)
    r = [np.repeat(np.arange(n), np.diff(base.ptr))]
    c = [base.col.astype(np.int64)]
    for h in hubs:
        others = rng.choice(n, size=350, replace=False)
        r += [np.full(350, h), others]
        c += [others, np.full(350, h)]
    return _csr_from_coo(n, n, np.concatenate(r), np.concatenate(c), rng)


def cop20k_like(seed: int = 6) -> CSR:
    """Random geometric graph on a 2-D grid, ~21.7 nnz/row."""
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
    return banded_random(5_154_859, 18.2, 300, far_frac=0.10, seed=seed)


SYNTH = {
    "cage4": cage4_like,
    "cant": cant_like,
    "webbase-1M": webbase_like,
    "mac_econ_fwd500": mac_econ_like,
    "scircuit": scircuit_like,
    "cop20k_A": cop20k_like,
    "cage15": cage15_like,
}


def matrix_path(name: str) -> Path | None:
    root = os.environ.get("MHS_MATRIX_DIR")
    if not root:
        return None
    p = Path(root) / name / f"{name}.mtx"
    return p if p.exists() else None


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
    return SYNTH[name](), f"synthetic:{name}-like"
