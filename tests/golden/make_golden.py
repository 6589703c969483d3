"""Generate the golden fixtures under tests/golden/ (run once, output committed).

The reference (yyssys/MH-SpGEMM) ships no tests, fixtures or golden vectors for
its SpGEMM path, and it cannot be built in this image (its kernels need nvcc,
its host code the CUDA runtime library).  The expected products below therefore
come from an INDEPENDENT implementation, scipy.sparse (SMMP), on small crafted
inputs with strictly positive values (no cancellation, so the structural
pattern the reference keeps equals scipy's numerical pattern).  scipy's
accumulation order (A entries in row order, then B entries in row order, one
multiply then one add) is exactly the order the oracle restates, so oracle vs
fixture is a bit-exact comparison.

Each case writes:
  <name>_A.mtx [<name>_B.mtx]   Matrix Market inputs (general real, 1-based)
  <name>.json                    {"M","N","ptr","col","val_hex"} of C = A*B
Matrix Market semantics cases (symmetric / pattern / integer / complex / skew /
duplicates / comments) store the expected CSR of the READ matrix instead
({"read": true, ...}), derived by hand from the reference rules
(inc/mmio_read.h:34-159) and cross-checked with scipy.io.mmread where scipy's
rules agree.

Usage: python tests/golden/make_golden.py
"""
from __future__ import annotations

import json
from pathlib import Path

import numpy as np
import scipy.sparse as sp

OUT = Path(__file__).resolve().parent


def write_mtx(path: Path, M, N, rows, cols, vals, field="real", symmetry="general", header_extra=()):
    lines = [f"%%MatrixMarket matrix coordinate {field} {symmetry}"]
    lines += list(header_extra)
    lines.append(f"{M} {N} {len(rows)}")
    for r, c, v in zip(rows, cols, vals):
        if field == "pattern":
            lines.append(f"{r + 1} {c + 1}")
        elif field == "integer":
            lines.append(f"{r + 1} {c + 1} {int(v)}")
        elif field == "complex":
            lines.append(f"{r + 1} {c + 1} {float(v[0])!r} {float(v[1])!r}")
        else:
            lines.append(f"{r + 1} {c + 1} {float(v)!r}")
    path.write_text("\n".join(lines) + "\n")


def csr_json(C: sp.csr_matrix, **extra):
    C = C.tocsr()
    C.sort_indices()
    return {"M": C.shape[0], "N": C.shape[1], "ptr": C.indptr.astype(int).tolist(),
            "col": C.indices.astype(int).tolist(), "val_hex": [float(x).hex() for x in C.data], **extra}


def product_case(name, A_rows, A_cols, A_vals, shapeA, B=None):
    M, K = shapeA
    write_mtx(OUT / f"{name}_A.mtx", M, K, A_rows, A_cols, A_vals)
    A = sp.csr_matrix((A_vals, (A_rows, A_cols)), shape=shapeA)
    # csr_matrix(coo) sums duplicates; keep the raw order instead for the product
    A = raw_csr(M, K, A_rows, A_cols, A_vals)
    if B is None:
        Bm = A
        bfile = None
    else:
        B_rows, B_cols, B_vals, shapeB = B
        write_mtx(OUT / f"{name}_B.mtx", shapeB[0], shapeB[1], B_rows, B_cols, B_vals)
        Bm = raw_csr(shapeB[0], shapeB[1], B_rows, B_cols, B_vals)
        bfile = f"{name}_B.mtx"
    C = A @ Bm
    C = C.tocsr()
    C.sort_indices()
    (OUT / f"{name}.json").write_text(json.dumps(csr_json(C, A=f"{name}_A.mtx", B=bfile)))


def raw_csr(M, N, rows, cols, vals):
    """CSR in the reader's layout: file order within a row, then sorted by
    (col, val) -- duplicates kept (inc/mmio_read.h:130-150)."""
    rows = np.asarray(rows, np.int64)
    cols = np.asarray(cols, np.int64)
    vals = np.asarray(vals, np.float64)
    order = np.lexsort((vals, cols, rows))
    rows, cols, vals = rows[order], cols[order], vals[order]
    ptr = np.zeros(M + 1, np.int64)
    np.cumsum(np.bincount(rows, minlength=M), out=ptr[1:])
    return sp.csr_matrix((vals, cols.astype(np.int32), ptr.astype(np.int32)), shape=(M, N))


def main():
    rng = np.random.default_rng(20261015)

    # cage4-shaped: 9x9, 49 nnz (diagonal + 40 off-diagonals)
    n = 9
    off = [(i, j) for i in range(n) for j in range(n) if i != j]
    pick = rng.choice(len(off), 40, replace=False)
    r = list(range(n)) + [off[k][0] for k in pick]
    c = list(range(n)) + [off[k][1] for k in pick]
    v = rng.uniform(0.1, 1.0, len(r))
    product_case("cage4_like", r, c, v, (n, n))

    # tile boundaries: columns 0,31,32,33,63,64,65,127,128 and a row spanning
    # several 64-column tiles, plus empty rows and single-entry rows
    n = 200
    rows, cols = [], []
    special = [0, 31, 32, 33, 63, 64, 65, 127, 128, 129, 191, 192, 199]
    for i in range(n):
        if i % 7 == 3:
            continue  # empty row
        if i % 11 == 5:
            rows.append(i); cols.append(int(rng.integers(0, n)))  # single entry
            continue
        k = int(rng.integers(1, 9))
        cs = set(rng.choice(special, size=min(k, len(special)), replace=False).tolist())
        cs |= set(rng.integers(0, n, size=k).tolist())
        for cc in sorted(cs):
            rows.append(i); cols.append(cc)
    vals = rng.uniform(0.1, 1.0, len(rows))
    product_case("tile_edges", rows, cols, vals, (n, n))

    # a dense row and a dense column (one C row and column become dense)
    n = 150
    rows = list(range(n)) + [7] * n + list(range(n))
    cols = list(range(n)) + list(range(n)) + [11] * n
    key = sorted(set(zip(rows, cols)))
    rows = [a for a, _ in key]; cols = [b for _, b in key]
    vals = rng.uniform(0.1, 1.0, len(rows))
    product_case("dense_row_col", rows, cols, vals, (n, n))

    # duplicates in A (same (i,k) twice) and in B rows: summed
    rows = [0, 0, 0, 1, 1, 2, 2, 2, 3]
    cols = [1, 1, 2, 0, 3, 2, 2, 3, 0]
    vals = [0.5, 0.25, 0.75, 1.0, 0.125, 0.5, 0.5, 2.0, 3.0]
    product_case("duplicates", rows, cols, vals, (4, 4))

    # rectangular A (30 x 500) * B (500 x 1000), B != A
    Ar = rng.integers(0, 30, 400); Ac = rng.integers(0, 500, 400)
    key = sorted(set(zip(Ar.tolist(), Ac.tolist())))
    Ar = [a for a, _ in key]; Ac = [b for _, b in key]
    Av = rng.uniform(0.1, 1.0, len(Ar))
    Br = rng.integers(0, 500, 3000); Bc = rng.integers(0, 1000, 3000)
    key = sorted(set(zip(Br.tolist(), Bc.tolist())))
    Br = [a for a, _ in key]; Bc = [b for _, b in key]
    Bv = rng.uniform(0.1, 1.0, len(Br))
    product_case("rect_AB", Ar, Ac, Av, (30, 500), B=(Br, Bc, Bv, (500, 1000)))

    # empty product: A has entries only into empty B rows
    product_case("empty_product", [0, 1], [2, 3], [1.0, 2.0], (4, 4),
                 B=([0, 1], [0, 1], [1.0, 1.0], (4, 4)))

    # ---- Matrix Market semantics (expected = the READ matrix) -------------
    def read_case(name, M, N, rows, cols, vals, field, symmetry, exp_rows, exp_cols, exp_vals,
                  header_extra=(), raw_text=None):
        if raw_text is None:
            write_mtx(OUT / f"{name}.mtx", M, N, rows, cols, vals, field, symmetry, header_extra)
        else:
            (OUT / f"{name}.mtx").write_text(raw_text)
        R = raw_csr(M, N, exp_rows, exp_cols, exp_vals)
        d = csr_json(R, read=True, file=f"{name}.mtx", is_symmetric=int(symmetry == "symmetric"))
        # csr_json sorts indices (stable for duplicates by value order already)
        (OUT / f"{name}.json").write_text(json.dumps(d))

    # symmetric: off-diagonals mirrored with the same value
    rows, cols, vals = [0, 2, 3, 3], [0, 0, 1, 3], [1.5, -2.0, 4.0, 0.5]
    er = rows + [0, 1]; ec = cols + [2, 3]; ev = vals + [-2.0, 4.0]
    read_case("mm_symmetric", 4, 4, rows, cols, vals, "real", "symmetric", er, ec, ev)
    # skew-symmetric: NOT mirrored (the reference only mirrors symmetric/hermitian)
    read_case("mm_skew", 4, 4, [1, 3], [0, 2], [2.0, -1.0], "real", "skew-symmetric",
              [1, 3], [0, 2], [2.0, -1.0])
    # hermitian complex: real part kept, mirrored with the SAME value
    read_case("mm_hermitian", 3, 3, [0, 2], [0, 1], [(1.0, 0.0), (2.5, -1.0)], "complex", "hermitian",
              [0, 2, 1], [0, 1, 2], [1.0, 2.5, 2.5])
    # pattern: value 1.0
    read_case("mm_pattern", 3, 5, [0, 1, 2, 2], [4, 0, 1, 3], [0, 0, 0, 0], "pattern", "general",
              [0, 1, 2, 2], [4, 0, 1, 3], [1.0, 1.0, 1.0, 1.0])
    # integer: converted to double
    read_case("mm_integer", 2, 2, [0, 1, 1], [1, 0, 1], [3, -7, 12], "integer", "general",
              [0, 1, 1], [1, 0, 1], [3.0, -7.0, 12.0])
    # duplicates kept, rows sorted by (col, val); comment lines; mixed-case banner
    text = ("%%MatrixMarket Matrix Coordinate Real General\n% a comment\n%another\n"
            "3 3 6\n1 3 5.0\n1 1 2.0\n1 3 -1.0\n3 2 0.25\n2 2 1e-3\n3 1 7\n")
    read_case("mm_dups_comments", 3, 3, None, None, None, "real", "general",
              [0, 0, 0, 2, 1, 2], [2, 0, 2, 1, 1, 0], [5.0, 2.0, -1.0, 0.25, 1e-3, 7.0], raw_text=text)
    print("golden fixtures written to", OUT)


if __name__ == "__main__":
    main()
