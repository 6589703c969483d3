"""CPU tests of the oracle (the checker) against the golden fixtures and known answers.

The oracle restates the reference host semantics (oracle/oracle.h cites the
file:line of each function).  These tests pin it: bit-exact against the
scipy-generated fixtures (tests/golden/, made by make_golden.py) and against
hand-derived answers.  No GPU involved.
"""
import numpy as np
import pytest

from oracle import oracle as orc
from _util import GOLDEN, PRODUCT_CASES, READ_CASES, load_golden, random_csr


@pytest.mark.parametrize("name", PRODUCT_CASES)
def test_oracle_product_matches_golden_bitexact(name):
    d, p, c, v = load_golden(name)
    M, K, Ap, Ai, Av, _ = orc.read_mtx(GOLDEN / d["A"])
    if d["B"]:
        _, N, Bp, Bi, Bv, _ = orc.read_mtx(GOLDEN / d["B"])
    else:
        N, Bp, Bi, Bv = K, Ap, Ai, Av
    Cp, Ci, Cv = orc.spgemm(Ap, Ai, Av, Bp, Bi, Bv, N)
    assert np.array_equal(Cp, p)
    assert np.array_equal(Ci, c)
    assert np.array_equal(Cv.view(np.uint64), v.view(np.uint64)), "values must be bit-identical"


@pytest.mark.parametrize("name", READ_CASES)
def test_oracle_mmio_matches_golden(name):
    d, p, c, v = load_golden(name)
    M, N, ptr, col, val, sym = orc.read_mtx(GOLDEN / d["file"])
    assert (M, N) == (d["M"], d["N"])
    assert np.array_equal(ptr, p) and np.array_equal(col, c)
    assert np.array_equal(val, v)
    assert sym == d["is_symmetric"]


def test_oracle_known_answer_2x2():
    # [[1,2],[0,3]]^2 = [[1,8],[0,9]]
    p = np.array([0, 2, 3], np.int32)
    c = np.array([0, 1, 1], np.int32)
    v = np.array([1.0, 2.0, 3.0])
    Cp, Ci, Cv = orc.spgemm(p, c, v, p, c, v, 2)
    assert Cp.tolist() == [0, 2, 3] and Ci.tolist() == [0, 1, 1] and Cv.tolist() == [1.0, 8.0, 9.0]


def test_oracle_keeps_structural_zeros():
    # [[1,1],[1,-1]]^2 = [[2,0],[0,2]]: the reference keeps the cancelled entries (nnz 4)
    p = np.array([0, 2, 4], np.int32)
    c = np.array([0, 1, 0, 1], np.int32)
    v = np.array([1.0, 1.0, 1.0, -1.0])
    Cp, Ci, Cv = orc.spgemm(p, c, v, p, c, v, 2)
    assert Cp.tolist() == [0, 2, 4] and Ci.tolist() == [0, 1, 0, 1]
    assert Cv.tolist() == [2.0, 0.0, 0.0, 2.0]


def test_oracle_flop_and_transpose():
    p, c, v = random_csr(300, 200, 5, seed=3)
    Bp, Bc, Bv = random_csr(200, 400, 4, seed=4)
    flop = orc.flop(c, Bp)
    assert flop == int(np.diff(Bp.astype(np.int64))[c].sum())
    T = orc.transpose(300, 200, p, c, v)
    assert T[0] == 200 and T[1] == 300
    import scipy.sparse as sp
    S = sp.csr_matrix((v, c, p), shape=(300, 200)).T.tocsr()
    S.sort_indices()
    assert np.array_equal(T[2], S.indptr) and np.array_equal(T[3], S.indices) and np.array_equal(T[4], S.data)


def test_oracle_vs_scipy_random_bitexact():
    import scipy.sparse as sp
    p, c, v = random_csr(2000, 1500, 8, seed=5)
    Bp, Bc, Bv = random_csr(1500, 3000, 6, seed=6)
    Cp, Ci, Cv = orc.spgemm(p, c, v, Bp, Bc, Bv, 3000)
    S = (sp.csr_matrix((v, c, p), shape=(2000, 1500)) @ sp.csr_matrix((Bv, Bc, Bp), shape=(1500, 3000))).tocsr()
    S.sort_indices()
    assert np.array_equal(Cp, S.indptr) and np.array_equal(Ci, S.indices)
    assert np.array_equal(Cv, S.data)


def test_oracle_row_subset_numeric():
    p, c, v = random_csr(500, 500, 6, seed=7)
    Cp, Ci, Cv = orc.spgemm(p, c, v, p, c, v, 500)
    Cp2 = orc.spgemm_symbolic(p, c, p, c, 500)
    Ci2 = np.full(Cp2[-1], -1, np.int32)
    Cv2 = np.zeros(Cp2[-1])
    orc.spgemm_numeric_rows(p, c, v, p, c, v, 500, Cp2, Ci2, Cv2, 100, 200)
    s, e = Cp2[100], Cp2[200]
    assert np.array_equal(Ci2[s:e], Ci[s:e]) and np.array_equal(Cv2[s:e], Cv[s:e])


def test_oracle_compare_ref_semantics():
    p = np.array([0, 2, 3], np.int32)
    c = np.array([0, 1, 1], np.int32)
    v = np.array([1.0, 2.0, 3.0])
    assert orc.compare_ref(p, c, v, p, c, v) == 1
    v2 = v.copy(); v2[1] += 1e-10      # |d| < 1e-9: accepted
    assert orc.compare_ref(p, c, v, p, c, v2) == 1
    v3 = v.copy(); v3[1] += 1e-6       # rejected
    assert orc.compare_ref(p, c, v, p, c, v3) == 0
    c4 = c.copy(); c4[0] = 1
    assert orc.compare_ref(p, c, v, p, c4, v) == 0
    # nnz mismatch -> the reference throws
    assert orc.compare_ref(p, c, v, np.array([0, 2, 2], np.int32), c[:2], v[:2]) == -1
    # > 10 errors -> throws
    P = np.arange(0, 41, 2, dtype=np.int32)
    C = np.tile(np.array([0, 1], np.int32), 20)
    V = np.ones(40)
    assert orc.compare_ref(P, C, V, P, C, V + 1.0) == -2


def test_oracle_compare_tol():
    p = np.array([0, 2, 3], np.int32)
    c = np.array([0, 1, 1], np.int32)
    v = np.array([1.0, 2.0, 3.0])
    assert orc.compare_tol(p, c, v, p, c, v * (1 + 5e-7)) == 0
    assert orc.compare_tol(p, c, v, p, c, v * (1 + 5e-6)) == 3
