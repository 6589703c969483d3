"""GPU parity: the HIP path (through the C-ABI) against the oracle.

Bar (BASELINE.json north_star): row_ptr and col_idx bit-exact; values within
1e-6 relative (|d| <= 1e-6*|ref| or |d| <= 1e-12), with the reference's own
1e-9 rule (src/CSR.cu:79-80) also checked where values are positive.  With
mixed-sign values (cancellation) the value tolerance is 1e-6 of the sum of
|a*b| of the entry, the pattern stays exact (structural zeros are kept).
"""
import os

import numpy as np
import pytest

import mhspgemm
from mhspgemm import synth
from oracle import oracle as orc
from _util import GOLDEN, PRODUCT_CASES, bin_zoo, group_zoo, load_golden, near_zoo, random_csr, run_zoo, tiny_zoo

pytestmark = pytest.mark.gpu

RTOL, ATOL = 1e-6, 1e-12


def run_gpu(tool, A, B):
    A.H2D(tool.device)
    if B is not A:
        B.H2D(tool.device)
    C, t = mhspgemm.spgemm(tool, A, B)
    try:
        p, c, v = C.to_host()
    finally:
        C.release()
    return p, c, v, t


def check(tool, A, B, ref_rule=True):
    p, c, v, t = run_gpu(tool, A, B)
    Cp, Ci, Cv = orc.spgemm(A.ptr, A.col, A.val, B.ptr, B.col, B.val, B.N)
    assert np.array_equal(p, Cp), "row_ptr must be bit-exact"
    assert np.array_equal(c, Ci), "col_idx must be bit-exact"
    ok, *_ = mhspgemm.compare_tol(Cp, Ci, Cv, p, c, v, RTOL, ATOL)
    assert ok, "values outside 1e-6 relative"
    if ref_rule:
        assert orc.compare_ref(Cp, Ci, Cv, p, c, v) == 1, "reference 1e-9 rule"
    assert t.nnzC == Cp[-1]
    assert t.flop == orc.flop(A.col, B.ptr)
    return t


@pytest.mark.parametrize("name", PRODUCT_CASES)
def test_golden_products(tool, name):
    d, gp, gc, gv = load_golden(name)
    A = mhspgemm.CSR()
    assert mhspgemm.readMtxFile(A, str(GOLDEN / d["A"])) == 0
    if d["B"]:
        B = mhspgemm.CSR()
        assert mhspgemm.readMtxFile(B, str(GOLDEN / d["B"])) == 0
    else:
        B = A
    p, c, v, t = run_gpu(tool, A, B)
    assert np.array_equal(p, gp) and np.array_equal(c, gc)
    ok, *_ = mhspgemm.compare_tol(gp, gc, gv, p, c, v, RTOL, ATOL)
    assert ok


def test_cage4_like(tool):
    A = synth.cage4_like()
    check(tool, A, A)


def test_cant_like_full(tool):
    A = synth.cant_like()
    t = check(tool, A, A)
    assert t.flop > 3e8


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_random_rect(tool, seed):
    p, c, v = random_csr(3000, 2000, 7, seed)
    Bp, Bc, Bv = random_csr(2000, 50_000, 12, seed + 100)
    A = mhspgemm.CSR(3000, 2000, p, c, v)
    B = mhspgemm.CSR(2000, 50_000, Bp, Bc, Bv)
    check(tool, A, B)


def test_bin_zoo_every_bin(tool):
    (M, K, Ap, Ac, Av), (K2, N, Bp, Bc, Bv) = bin_zoo()
    A = mhspgemm.CSR(M, K, Ap, Ac, Av)
    B = mhspgemm.CSR(K2, N, Bp, Bc, Bv)
    t = check(tool, A, B)
    # every symbolic bin (1..4, 11: 10 KiB wave) and numeric bin (3..5: block and global kernels,
    # 12/13: 64-lane sort classes for scattered rows, 14/15: hash-mode wave kernels) saw rows
    assert all(t.sym_bins[i] > 0 for i in (0, 1, 2, 3, 4, 11)), t.sym_bins
    assert all(t.num_bins[i] > 0 for i in (0, 3, 4, 5, 12, 13, 14, 15)), t.num_bins


@pytest.mark.parametrize("seed", [7, 8])
def test_tiny_zoo_every_class(tool, seed):
    (M, K, Ap, Ac, Av), (K2, N, Bp, Bc, Bv) = tiny_zoo(seed)
    A = mhspgemm.CSR(M, K, Ap, Ac, Av)
    B = mhspgemm.CSR(K2, N, Bp, Bc, Bv)
    t = check(tool, A, B)
    # every small tiny class (symbolic bins 5..8, numeric bins 8..11) and the wave bins saw rows
    assert all(t.sym_bins[i] > 0 for i in range(5, 9)), t.sym_bins
    assert all(t.num_bins[i] > 0 for i in range(8, 12)), t.num_bins
    assert t.num_bins[1] + t.num_bins[14] > 0, t.num_bins


@pytest.mark.parametrize("seed", [5, 6])
def test_run_zoo_same_pattern_rows(tool, seed):
    (M, K, Ap, Ac, Av), (K2, N, Bp, Bc, Bv) = run_zoo(seed)
    A = mhspgemm.CSR(M, K, Ap, Ac, Av)
    B = mhspgemm.CSR(K2, N, Bp, Bc, Bv)
    t = check(tool, A, B)
    assert t.num_bins[1] + t.num_bins[14] > 0 and t.num_bins[3] > 0, t.num_bins  # wave and block kernels saw rows


@pytest.mark.parametrize("seed", [3, 4])
def test_group_zoo_row_groups(tool, seed):
    (M, K, Ap, Ac, Av), (K2, N, Bp, Bc, Bv) = group_zoo(seed)
    A = mhspgemm.CSR(M, K, Ap, Ac, Av)
    B = mhspgemm.CSR(K2, N, Bp, Bc, Bv)
    t = check(tool, A, B)
    assert t.num_bins[6] > 0, t.num_bins  # grouped wave bin used


def test_row_groups_off_matches(tool, monkeypatch):
    # the same product with row groups disabled (MHS_NO_GROUPS, read at context creation)
    (M, K, Ap, Ac, Av), (K2, N, Bp, Bc, Bv) = group_zoo(5)
    A = mhspgemm.CSR(M, K, Ap, Ac, Av)
    B = mhspgemm.CSR(K2, N, Bp, Bc, Bv)
    monkeypatch.setenv("MHS_NO_GROUPS", "1")
    plain = mhspgemm.Tool(tool.device)
    try:
        t = check(plain, A, B)
        assert t.num_bins[6] == 0 and t.num_bins[7] == 0, t.num_bins
    finally:
        plain.close()


@pytest.mark.parametrize("near", [True, False])
def test_near_row_groups(tool, near, monkeypatch):
    """Near row groups (GRP_NEAR): dof triples whose A rows differ by dropped entries run
    as row groups over their union row once k_near has found their C patterns equal;
    rows whose patterns differ (an appended far column), duplicate and unsorted A
    columns stay exact.  MHS_NO_NEAR=1 (read at context creation): every such row alone."""
    (M, K, Ap, Ac, Av), (K2, N, Bp, Bc, Bv) = near_zoo()
    A = mhspgemm.CSR(M, K, Ap, Ac, Av)
    B = mhspgemm.CSR(K2, N, Bp, Bc, Bv)
    if not near:
        monkeypatch.setenv("MHS_NO_NEAR", "1")
    t2 = mhspgemm.Tool(tool.device)
    try:
        t = check(t2, A, B, ref_rule=False)
        grouped = t.num_bins[6] + t.num_bins[7]
        if near:
            assert grouped > M // 10, t.num_bins
        else:
            assert grouped < M // 30, t.num_bins
    finally:
        t2.close()


def test_cant_perturbed_near_groups(tool):
    """cant-perturbed (3 % of the entries dropped): its dof triples run as near groups."""
    A = synth.cant_perturbed()
    t = check(tool, A, A)
    assert t.num_bins[6] + t.num_bins[7] > A.M // 5, t.num_bins


def _perturbed_fem(nx, ny, nz, drop, seed):
    A = synth.fem_grid(nx, ny, nz, 3, seed=seed)
    rng = np.random.default_rng(seed + 1000)
    rows = np.repeat(np.arange(A.M, dtype=np.int64), np.diff(A.ptr))
    keep = (rows == A.col) | (rng.random(A.nnz) >= drop)
    ptr = np.zeros(A.M + 1, np.int64)
    np.cumsum(np.bincount(rows[keep], minlength=A.M), out=ptr[1:])
    return mhspgemm.CSR(A.M, A.N, ptr.astype(np.int32), A.col[keep].copy(), A.val[keep].copy())


@pytest.mark.parametrize("drop", [0.01, 0.03, 0.08])
def test_near_union_runs_square(tool, drop):
    """A*A with near row groups: B's near groups walk their union rows as runs where the A
    row holds the whole group (finish_chunk), and as single rows where a drop broke the
    group in the A row.  The same product with B an unaliased copy of A (no union runs)
    must agree with the oracle too."""
    A = _perturbed_fem(7, 6, 24, drop, seed=int(drop * 1000))
    t = check(tool, A, A)
    assert t.num_bins[6] + t.num_bins[7] > 0, t.num_bins
    B = mhspgemm.CSR(A.M, A.N, A.ptr.copy(), A.col.copy(), A.val.copy())
    check(tool, A, B)


def test_near_groups_nonfinite_values(tool):
    """Near groups and union runs add explicit 0*b / a*0 products, which turn into NaN when
    b or a is Inf / NaN, where the reference (src/CSR.cu:48-96 compares every entry) never
    forms the product.  k_mask_b checks B's values (A's, when B is A) and a non-finite
    value turns near groups off for the call: Inf and NaN land exactly where the oracle has
    them, A*A and A*B with B an unaliased copy."""
    A0 = _perturbed_fem(7, 6, 24, 0.03, seed=31)
    v = A0.val.copy()
    v[[5, 1000, 2500, 7001]] = np.inf
    v[777] = -np.inf
    v[4321] = np.nan
    A = mhspgemm.CSR(A0.M, A0.N, A0.ptr, A0.col, v)
    for B in (A, mhspgemm.CSR(A.M, A.N, A.ptr.copy(), A.col.copy(), A.val.copy())):
        p, c, vv, t = run_gpu(tool, A, B)
        Cp, Ci, Cv = orc.spgemm(A.ptr, A.col, A.val, B.ptr, B.col, B.val, B.N)
        assert np.array_equal(p, Cp) and np.array_equal(c, Ci)
        assert np.array_equal(np.isnan(vv), np.isnan(Cv)), "NaN positions differ"
        assert np.array_equal(np.isposinf(vv), np.isposinf(Cv)) and np.array_equal(np.isneginf(vv), np.isneginf(Cv))
        fin = np.isfinite(Cv)
        assert fin.sum() > len(Cv) // 2
        assert np.allclose(vv[fin], Cv[fin], rtol=RTOL, atol=ATOL)
    # the finite product of the same pattern does run near groups (the switch is per call)
    t = check(tool, A0, A0)
    assert t.num_bins[6] + t.num_bins[7] > 0, t.num_bins


def test_fem_dof_runs_square(tool):
    # A*A with dof 1..4 per node: runs of every length up to and past the merge cap
    for dof in (1, 2, 3, 4, 6):
        A = synth.fem_grid(5, 4, 9, dof=dof)
        check(tool, A, A)


def test_unsynced_calls_and_numeric_event_ring(tool):
    from mhspgemm import _lib as L
    A = synth.fem_grid(6, 5, 12)
    A.H2D(tool.device)
    Cp, Ci, Cv = orc.spgemm(A.ptr, A.col, A.val, A.ptr, A.col, A.val, A.N)
    tool.set_option(L.MHS_OPT_SYNC, 0)
    tool.set_option(L.MHS_OPT_NUMERIC_EVENTS, 4)
    try:
        outs = [mhspgemm.spgemm(tool, A, A, timing=False)[0] for _ in range(6)]
        for C in outs:  # each result intact although the calls never waited
            p, c, v = C.to_host()
            assert np.array_equal(p, Cp) and np.array_equal(c, Ci)
            assert mhspgemm.compare_tol(Cp, Ci, Cv, p, c, v, RTOL, ATOL)[0]
            C.release()
        ms = tool.numeric_ms(10)
        assert len(ms) == 4 and all(m > 0 for m in ms), ms
    finally:
        tool.set_option(L.MHS_OPT_SYNC, 1)
        tool.set_option(L.MHS_OPT_NUMERIC_EVENTS, 0)
    with pytest.raises(mhspgemm.MHSpGEMMError):
        tool.set_option(99, 1)


def test_mixed_sign_cancellation_keeps_structure(tool):
    p, c, v = random_csr(1500, 1500, 10, seed=9, signed=True)
    A = mhspgemm.CSR(1500, 1500, p, c, v)
    gp, gc, gv, _ = run_gpu(tool, A, A)
    Cp, Ci, Cv = orc.spgemm(p, c, v, p, c, v, 1500)
    assert np.array_equal(gp, Cp) and np.array_equal(gc, Ci)
    # tolerance scaled by sum |a*b| per entry
    _, _, absv = orc.spgemm(p, c, np.abs(v), p, c, np.abs(v), 1500)
    assert np.all(np.abs(gv - Cv) <= 1e-6 * absv + 1e-300)


def test_exact_cancellation_structural_zero(tool):
    p = np.array([0, 2, 4], np.int32)
    c = np.array([0, 1, 0, 1], np.int32)
    v = np.array([1.0, 1.0, 1.0, -1.0])
    A = mhspgemm.CSR(2, 2, p, c, v)
    gp, gc, gv, _ = run_gpu(tool, A, A)
    assert gp.tolist() == [0, 2, 4] and gc.tolist() == [0, 1, 0, 1]
    assert gv.tolist() == [2.0, 0.0, 0.0, 2.0]


def test_empty_and_degenerate(tool):
    # all-empty rows
    A = mhspgemm.CSR(5, 5, np.zeros(6, np.int32), np.zeros(0, np.int32), np.zeros(0))
    p, c, v, t = run_gpu(tool, A, A)
    assert p.tolist() == [0] * 6 and len(c) == 0
    # 1x1
    A = mhspgemm.CSR(1, 1, np.array([0, 1], np.int32), np.array([0], np.int32), np.array([3.0]))
    p, c, v, t = run_gpu(tool, A, A)
    assert p.tolist() == [0, 1] and c.tolist() == [0] and v.tolist() == [9.0]


def test_error_unsorted_B(tool):
    p = np.array([0, 2, 3], np.int32)
    c = np.array([1, 0, 1], np.int32)  # row 0 unsorted
    A = mhspgemm.CSR(2, 2, p, c, np.ones(3))
    A.H2D(tool.device)
    with pytest.raises(mhspgemm.MHSpGEMMError) as e:
        mhspgemm.spgemm(tool, A, A)
    assert e.value.status == 3 and "sorted" in str(e.value)


def test_error_dimension_mismatch(tool):
    A = mhspgemm.CSR(2, 3, np.array([0, 1, 2], np.int32), np.array([0, 2], np.int32), np.ones(2))
    A.H2D(tool.device)
    with pytest.raises(mhspgemm.MHSpGEMMError) as e:
        mhspgemm.spgemm(tool, A, A)
    assert e.value.status == 3


def test_error_column_out_of_range(tool):
    A = mhspgemm.CSR(2, 2, np.array([0, 1, 2], np.int32), np.array([0, 5], np.int32), np.ones(2))
    A.H2D(tool.device)
    with pytest.raises(mhspgemm.MHSpGEMMError):
        mhspgemm.spgemm(tool, A, A)


@pytest.mark.parametrize("long_row", [False, True])
def test_error_column_out_of_range_mixed_row(tool, long_row):
    # a row mixing valid and out-of-range columns: the row must enter no
    # symbolic bin (its kernels gather bmeta[Acol[j]] unchecked) and the call must
    # return MHS_ERR_INVALID; the context stays usable afterwards
    if long_row:
        Bp, Bc, Bv = random_csr(50, 3000, 100, seed=21)
        cols = list(range(0, 40)) + [77]  # 40 valid B rows (~4000 products: a wave bin) + 1 bad
        Ap = np.array([0, len(cols), len(cols) + 2], np.int32)
        Ac = np.array(cols + [1, 2], np.int32)
        A = mhspgemm.CSR(2, 50, Ap, Ac, np.ones(len(Ac)))
        B = mhspgemm.CSR(50, 3000, Bp, Bc, Bv)
    else:
        A = mhspgemm.CSR(2, 2, np.array([0, 2, 2], np.int32), np.array([0, 5], np.int32), np.ones(2))
        B = mhspgemm.CSR(2, 2, np.array([0, 1, 2], np.int32), np.array([0, 1], np.int32), np.ones(2))
    A.H2D(tool.device)
    B.H2D(tool.device)
    with pytest.raises(mhspgemm.MHSpGEMMError) as e:
        mhspgemm.spgemm(tool, A, B)
    assert e.value.status == 3 and "A column" in str(e.value)
    check(tool, synth.cage4_like(), synth.cage4_like())


def test_repeat_calls_reuse_workspace(tool):
    A = synth.cage4_like()
    A.H2D(tool.device)
    ref = None
    for _ in range(5):
        C, _ = mhspgemm.spgemm(tool, A, A, timing=False)
        got = C.to_host()
        C.release()
        if ref is None:
            ref = got
        assert all(np.array_equal(x, y) for x, y in zip(ref[:2], got[:2]))


def test_mirror_interface_MH_spgemm(tool):
    A = synth.cage4_like()
    B = A
    A.H2D(tool.device)
    C = mhspgemm.CSR()
    timing = mhspgemm.Timing()
    mhspgemm.MH_spgemm(A, B, C, timing, tool)
    C.D2H()
    Cp, Ci, Cv = orc.spgemm(A.ptr, A.col, A.val, A.ptr, A.col, A.val, A.N)
    ref = mhspgemm.CSR(A.M, A.N, Cp, Ci, Cv)
    assert C == ref
    assert timing.getTotal() > 0 and timing.flop == orc.flop(A.col, A.ptr)
    C.d_release_csr()


@pytest.mark.slow
@pytest.mark.parametrize("name", ["webbase-1M", "mac_econ_fwd500", "scircuit", "cop20k_A",
                                  # the headline's robustness variants (broken dof runs)
                                  "cant-s1", "cant-perturbed",
                                  # the rest of 16matrix.txt (stand-ins, synth.py)
                                  "pdb1HYS", "pwtk", "cage12", "hood", "rma10", "shipsec1", "offshore"])
def test_baseline_configs_full(tool, name):
    A = synth.SYNTH[name]()
    check(tool, A, A)
    A.d_release_csr()


@pytest.mark.slow
@pytest.mark.parametrize("name", ["wb-edu", "GAP-road", "delaunay_n24"])
def test_huge_m_full(tool, name):
    """16matrix.txt's huge-M, few-entries-per-row stand-ins (9.8 M - 24 M rows), whole
    matrix against the oracle: row_ptr / col_idx bit-exact, values within 1e-6."""
    A = synth.SYNTH[name]()
    check(tool, A, A, ref_rule=False)
    A.d_release_csr()


@pytest.mark.slow
def test_cage15_like_whole_matrix(tool):
    """Full-size cage15-like (5.15 M rows, 1.56 G entries of C), EVERY row against the
    oracle -- the reference's CHECK_RESULT compares all of C (src/main.cu:187-199,
    src/CSR.cu:48-96): row blocks of 500 k rows, each block's C col / val slice copied
    from the device and compared with the oracle's product of the same rows of A with
    the whole B (row_ptr and col_idx bit-exact, values within 1e-6 relative)."""
    import ctypes
    from mhspgemm import _lib as L
    A = synth.cage15_like()
    A.H2D(tool.device)
    C, t = mhspgemm.spgemm(tool, A, A)
    try:
        assert t.flop == orc.flop(A.col, A.ptr)
        lib, ctx = L.lib(), tool.ctx
        p = np.empty(A.M + 1, np.int32)
        assert lib.mhs_memcpy(ctx, p.ctypes.data, C.c.ptr, p.nbytes, 1) == 0
        assert p[-1] == t.nnzC == C.nnz
        step = 500_000
        for r0 in range(0, A.M, step):
            r1 = min(A.M, r0 + step)
            a0, a1 = int(A.ptr[r0]), int(A.ptr[r1])
            Sp = (A.ptr[r0:r1 + 1] - a0).astype(np.int32)
            Cp, Ci, Cv = orc.spgemm(Sp, A.col[a0:a1], A.val[a0:a1], A.ptr, A.col, A.val, A.N)
            c0, c1 = int(p[r0]), int(p[r1])
            gp = (p[r0:r1 + 1] - c0).astype(np.int32)
            assert np.array_equal(gp, Cp), f"row_ptr of rows [{r0}, {r1})"
            gc = np.empty(c1 - c0, np.int32)
            gv = np.empty(c1 - c0, np.float64)
            if c1 > c0:
                assert lib.mhs_memcpy(ctx, gc.ctypes.data, ctypes.c_void_p(C.c.col + 4 * c0), gc.nbytes, 1) == 0
                assert lib.mhs_memcpy(ctx, gv.ctypes.data, ctypes.c_void_p(C.c.val + 8 * c0), gv.nbytes, 1) == 0
            bad = orc.compare_tol(Cp, Ci, Cv, gp, gc, gv, RTOL, ATOL)
            assert bad == 0, f"rows [{r0}, {r1}): {bad} entries differ (col exact, val 1e-6)"
    finally:
        C.release()
        A.d_release_csr()


# ----------------------------------------------- AAT mode and vendor cross-check ---

@pytest.mark.parametrize("shape", [(700, 1900, 6), (2500, 300, 9), (1, 1, 1)])
def test_device_transpose_bit_exact(tool, shape):
    # mhs_transpose vs the oracle's restatement of src/utils.cpp:20-46
    M, N, per = shape
    p, c, v = random_csr(M, N, per, seed=M + N)
    A = mhspgemm.CSR(M, N, p, c, v)
    A.H2D(tool.device)
    T = mhspgemm.transpose(tool, A)
    tp, tc, tv = T.dev.to_host()
    T.d_release_csr()
    oM, oN, op, oc, ov = orc.transpose(M, N, p, c, v)
    assert (T.M, T.N) == (N, M) == (oM, oN)
    assert np.array_equal(tp, op) and np.array_equal(tc, oc) and np.array_equal(tv, ov)


@pytest.mark.parametrize("shape", [(1200, 5000, 7), (3000, 800, 12)])
def test_aat_rectangular(tool, shape):
    # AAT=1 (inc/common.h:37, src/main.cu:98-99): C = A * A^T for a non-square A
    M, N, per = shape
    p, c, v = random_csr(M, N, per, seed=N)
    A = mhspgemm.CSR(M, N, p, c, v)
    A.H2D(tool.device)
    B = mhspgemm.transpose(tool, A)
    bp, bc, bv = B.dev.to_host()
    Bh = mhspgemm.CSR(N, M, bp, bc, bv)
    t = check(tool, A, Bh)
    assert t.nnzC > 0
    B.d_release_csr()


@pytest.mark.parametrize("which", ["cage4", "cant", "scircuit", "rect"])
def test_rocsparse_crosscheck(tool, which):
    # CUSPARSE + CHECK_RESULT (src/main.cu:148-199): the vendor's C equals ours under
    # CSR::operator== (pattern exact, values by the reference rule)
    if which == "rect":
        p, c, v = random_csr(3000, 2000, 7, 1)
        Bp, Bc, Bv = random_csr(2000, 50_000, 12, 101)
        A, B = mhspgemm.CSR(3000, 2000, p, c, v), mhspgemm.CSR(2000, 50_000, Bp, Bc, Bv)
    else:
        A = synth.SYNTH[which]()
        B = A
    p, c, v, t = run_gpu(tool, A, B)
    V, ms = mhspgemm.vendor_spgemm(tool, A, B)
    vp, vc, vv = V.to_host()
    V.release()
    assert ms > 0
    assert np.array_equal(p, vp) and np.array_equal(c, vc)
    ok, *_ = mhspgemm.compare_tol(vp, vc, vv, p, c, v, RTOL, ATOL)
    assert ok


def test_wide_column_space_small_rows(tool):
    # N > 2^23: the numeric tiny classes pack a column's offset from the row's first tile
    # into 23 bits, so rows over a narrow span still sort in registers (symbolic sorted them
    # too: no cached tile masks), at column indices past 2^23
    p, c, v = random_csr(3000, 400, 4, seed=12)
    A = mhspgemm.CSR(3000, 400, p, c, v)
    Bp, Bc, Bv = random_csr(400, 1500, 6, seed=13)
    Bc = (Bc + 8_600_000).astype(np.int32)  # every column past 2^23, within ~24 tiles
    B = mhspgemm.CSR(400, 9_000_000, Bp, Bc, Bv)
    t = check(tool, A, B)
    assert t.sym_bins[5] + t.sym_bins[6] > 0, t.sym_bins
    assert sum(t.num_bins[8:12]) > 0, t.num_bins


def test_tiny_rows_spanning_past_key_range(tool):
    # tiny rows whose columns span more than 2^23 (first column near 0, last near 9 M):
    # their offsets do not fit the packed sort keys, so numeric runs them with tables
    K, N = 400, 9_000_000
    rng = np.random.default_rng(5)
    Bp = np.arange(0, 2 * K + 1, 2, dtype=np.int32)
    Bc = np.stack([np.arange(K) * 3, 8_900_000 + np.arange(K)], 1).reshape(-1).astype(np.int32)
    B = mhspgemm.CSR(K, N, Bp, Bc, rng.uniform(0.5, 1.5, 2 * K))
    p, c, v = random_csr(2000, K, 3, seed=6)
    A = mhspgemm.CSR(2000, K, p, c, v)
    t = check(tool, A, B)
    assert sum(t.num_bins[8:14]) == 0, t.num_bins


@pytest.mark.parametrize("per_b", [16, 20])
def test_block_hash_rows_rank(tool, per_b):
    # hashed rows with ~1000 tiles over a moderate span: the 256-thread kernel ranks the
    # tiles by a bitmap over the span instead of sorting them
    rng = np.random.default_rng(per_b)
    K, N = 2000, 200_000
    Bp, Bc, Bv = random_csr(K, N, 50, seed=per_b + 1)
    rows = [np.sort(rng.choice(K, per_b, replace=False)) for _ in range(300)]
    Ap = np.zeros(len(rows) + 1, np.int64)
    Ap[1:] = np.cumsum([len(r) for r in rows])
    A = mhspgemm.CSR(len(rows), K, Ap.astype(np.int32), np.concatenate(rows).astype(np.int32),
                     rng.uniform(0.1, 1.0, int(Ap[-1])))
    B = mhspgemm.CSR(K, N, Bp, Bc, Bv)
    t = check(tool, A, B)
    assert t.num_bins[3] > 0, t.num_bins


@pytest.mark.parametrize("spread", [1, 40])
def test_wide_symbolic_rows_few_tiles(tool, spread):
    # rows with thousands of tile products over a ~31 k-tile span but only a few distinct
    # tiles: symbolic counts them as wide rows (dense windows, two of them), numeric hashes
    # them from the tile list symbolic leaves -- the list must span the windows
    K, N = 3000, 2_000_000
    k = np.arange(K)
    first = (k % spread) * 50_000 + (k % 7)
    last = 1_999_000 + (k % 64)
    Bp = np.arange(0, 2 * K + 1, 2, dtype=np.int32)
    Bc = np.stack([first, last], 1).reshape(-1).astype(np.int32)
    rng = np.random.default_rng(spread)
    B = mhspgemm.CSR(K, N, Bp, Bc, rng.uniform(0.5, 1.5, 2 * K))
    rows = [np.arange(K)] * 3 + [np.sort(rng.choice(K, 2000, replace=False)) for _ in range(3)]
    Ap = np.zeros(len(rows) + 1, np.int64)
    Ap[1:] = np.cumsum([len(r) for r in rows])
    A = mhspgemm.CSR(len(rows), K, Ap.astype(np.int32), np.concatenate(rows).astype(np.int32),
                     rng.uniform(0.1, 1.0, int(Ap[-1])))
    t = check(tool, A, B)
    assert t.sym_bins[3] + t.sym_bins[4] > 0, t.sym_bins


@pytest.mark.parametrize("case", ["ranked", "wide"])
def test_hub_rows_span_rank_and_windows(tool, case):
    # hub rows (thousands of A entries on short scattered B rows): "ranked" -- a few thousand
    # distinct tiles over a ~100 k-tile span, past the 256-thread hash budget: symbolic and
    # numeric rank tiles by a span bitmap in the 1024-thread kernels; "wide" -- ~9 k tiles over
    # a ~940 k-tile span, whose bitmap does not fit: symbolic walks windows, numeric accumulates
    # in C with global atomics
    rng = np.random.default_rng(31)
    K, N, per = (3000, 6_400_000, 2) if case == "ranked" else (3000, 60_000_000, 3)
    Bl = np.full(K, per)
    Bp = np.zeros(K + 1, np.int32)
    Bp[1:] = np.cumsum(Bl)
    Bc = np.concatenate([np.sort(rng.choice(N, per, replace=False)) for _ in range(K)]).astype(np.int32)
    B = mhspgemm.CSR(K, N, Bp, Bc, rng.uniform(0.5, 1.5, int(Bp[-1])))
    rows = [np.sort(rng.choice(K, 2500 if case == "ranked" else K, replace=False)) for _ in range(6)]
    rows += [np.sort(rng.choice(K, 4, replace=False)) for _ in range(50)]  # small rows beside them
    Ap = np.zeros(len(rows) + 1, np.int64)
    Ap[1:] = np.cumsum([len(r) for r in rows])
    A = mhspgemm.CSR(len(rows), K, Ap.astype(np.int32), np.concatenate(rows).astype(np.int32),
                     rng.uniform(0.1, 1.0, int(Ap[-1])))
    t = check(tool, A, B)
    assert t.num_bins[4] >= 6, t.num_bins  # the hub rows run in the 1024-thread kernel


def test_oom_row_chunked_fallback(tool):
    # SURVEY §5 fallback: a context whose memory budget holds C but not C beside the full
    # workspace runs the product row-chunked (workspace for a quarter of the rows here);
    # the result is the same C
    from mhspgemm import _lib as L
    A = synth.cant_like()
    A.H2D(tool.device)
    small = mhspgemm.Tool(tool.device)
    try:
        small.set_option(L.MHS_OPT_MEM_BUDGET, 300)  # MiB: C is 210 MB, the workspace ~170 MB without near groups (~380 MB with them: dropped first)
        C, t = mhspgemm.spgemm(small, A, A)
        p, c, v = C.to_host()
        C.release()
        assert small.chunked_calls() == 1
        Cp, Ci, Cv = orc.spgemm(A.ptr, A.col, A.val, A.ptr, A.col, A.val, A.N)
        assert np.array_equal(p, Cp) and np.array_equal(c, Ci)
        assert mhspgemm.compare_tol(Cp, Ci, Cv, p, c, v, RTOL, ATOL)[0]
        assert t.nnzC == Cp[-1] and t.flop == orc.flop(A.col, A.ptr)
        # C alone beyond the budget: MHS_ERR_OOM right after the counting pass (the
        # size of C does not depend on the chunking, so no halving down to one-row chunks)
        import time
        small.set_option(L.MHS_OPT_MEM_BUDGET, 150)
        t0 = time.perf_counter()
        with pytest.raises(mhspgemm.MHSpGEMMError) as e:
            mhspgemm.spgemm(small, A, A)
        assert e.value.status == 2 and "C itself" in str(e.value)
        assert time.perf_counter() - t0 < 3.0
    finally:
        small.close()


def test_oom_one_row_chunks(tool, monkeypatch):
    # when the counting pass only fits one-row chunks, the second pass must try the
    # one-row workspace beside C too.  A 100 000-tile row-cache slot (1.2 MB a row) makes a
    # 2-row workspace exceed a 2 MiB budget while a 1-row one fits; C is a few KB.
    from mhspgemm import _lib as L
    monkeypatch.setenv("MHS_MC_LIST", "100000")
    monkeypatch.setenv("MHS_SPILL_CAP", "1024")
    small = mhspgemm.Tool(tool.device)
    try:
        p, c, v = random_csr(24, 40, 3, seed=11)
        Bp, Bc, Bv = random_csr(40, 30, 2, seed=12)
        A = mhspgemm.CSR(24, 40, p, c, v)
        B = mhspgemm.CSR(40, 30, Bp, Bc, Bv)
        small.set_option(L.MHS_OPT_MEM_BUDGET, 2)
        t = check(small, A, B)
        assert small.chunked_calls() == 1 and t.nnzC > 0
    finally:
        small.close()


def test_probe_conflict_counter():
    # the reference's HASH_CONFLICT diagnostic (inc/common.h:18, src/main.cu:68-71): the probe
    # build counts conflicts of the hashed tile tables; the product library refuses the query
    import subprocess
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parent.parent
    code = (
        "import sys; sys.path[:0] = [%r, %r]\n"
        "import mhspgemm\n"
        "from mhspgemm import synth\n"
        "A = synth.SYNTH['cop20k_A']()\n"
        "A.H2D(0)\n"
        "t = mhspgemm.Tool(0)\n"
        "try:\n"
        "    t.probe_conflicts()\n"
        "except mhspgemm.MHSpGEMMError as e:\n"
        "    print('REFUSED', e.status)\n"
        "C, _ = mhspgemm.spgemm(t, A, A); C.release()\n"
        "print('CONFLICTS', t.probe_conflicts(), t.probe_conflicts())\n"
    ) % (str(root), str(root / "mh-spgemm_amd"))
    env = dict(os.environ)
    env["MHS_LIB"] = str(root / "mh-spgemm_amd" / "mhspgemm" / "libmhspgemm_probe.so")
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    line = [l for l in out.stdout.splitlines() if l.startswith("CONFLICTS")][0].split()
    assert int(line[1]) > 0 and int(line[2]) == 0, line  # counted, then reset by the query
    env.pop("MHS_LIB")
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240)
    assert "REFUSED 3" in out.stdout, out.stdout + out.stderr[-2000:]


@pytest.mark.parametrize("cap", [None, "300"])
def test_spill_lists_and_full_region(tool, cap, monkeypatch):
    # rows with more tiles than the row-cache slot (here a 16-tile slot) hand their tile list
    # to numeric through the spill region; with a 300-entry region most rows find it full
    # (lofs = -1) and numeric walks their tiles again -- same C either way
    if cap:
        monkeypatch.setenv("MHS_SPILL_CAP", cap)
    monkeypatch.setenv("MHS_MC_LIST", "16")
    t2 = mhspgemm.Tool(tool.device)
    try:
        A = synth.SYNTH["webbase-1M"]() if cap is None else synth.scircuit_like()
        check(t2, A, A, ref_rule=cap is not None)
        (M, K, Ap, Ac, Av), (K2, N, Bp, Bc, Bv) = bin_zoo()
        check(t2, mhspgemm.CSR(M, K, Ap, Ac, Av), mhspgemm.CSR(K2, N, Bp, Bc, Bv))
    finally:
        t2.close()


@pytest.mark.parametrize("slots", [True, False])
def test_numeric_first_tiny_rows(tool, slots, monkeypatch):
    # numeric-first tiny rows (probed from 512 K rows; here for every size): symbolic sorts
    # them in the numeric classes and sums them into value slots, numeric copies the slots
    # into C.  Without slots (no room, or too many other rows) the probe falls back to the
    # usual bin lists.  Rows spanning past the packed-key range and row groups stay on
    # their usual paths.
    if not slots:
        monkeypatch.setenv("MHS_NFT_NO_SLOTS", "1")
    monkeypatch.setenv("MHS_NFT_OTHER_PCT", "100")  # slots whatever the share of other rows
    t2 = mhspgemm.Tool(tool.device)
    try:
        t2.set_option(mhspgemm._lib.MHS_OPT_TINY_FIRST_ROWS, 0)
        for seed in (7, 8):
            (M, K, Ap, Ac, Av), (K2, N, Bp, Bc, Bv) = tiny_zoo(seed)
            t = check(t2, mhspgemm.CSR(M, K, Ap, Ac, Av), mhspgemm.CSR(K2, N, Bp, Bc, Bv))
            assert all(t.sym_bins[i] > 0 for i in range(5, 9)), t.sym_bins
            # numeric's class lists: copied from the slots, or sorted again without them
            assert all(t.num_bins[i] > 0 for i in range(8, 12)), t.num_bins
        (M, K, Ap, Ac, Av), (K2, N, Bp, Bc, Bv) = group_zoo(3)
        check(t2, mhspgemm.CSR(M, K, Ap, Ac, Av), mhspgemm.CSR(K2, N, Bp, Bc, Bv))
        # tiny rows past the 2^23-column key range: tables in both phases
        K, N = 400, 9_000_000
        rng = np.random.default_rng(5)
        Bp = np.arange(0, 2 * K + 1, 2, dtype=np.int32)
        Bc = np.stack([np.arange(K) * 3, 8_900_000 + np.arange(K)], 1).reshape(-1).astype(np.int32)
        p, c, v = random_csr(2000, K, 3, seed=6)
        t = check(t2, mhspgemm.CSR(2000, K, p, c, v), mhspgemm.CSR(K, N, Bp, Bc, rng.uniform(0.5, 1.5, 2 * K)))
        assert sum(t.num_bins[8:14]) == 0, t.num_bins  # (no candidates: the probe keeps the usual lists)
        for name in ("scircuit", "webbase-1M", "cant"):
            A = synth.SYNTH[name]()
            check(t2, A, A)
            A.d_release_csr()
    finally:
        t2.close()



# ---- round 5: path counters (mhs_ctx_stat) assert that the rarer paths actually ran ----------

def test_split_block_bins_ran(tool):
    """block bins split by LDS need (k_split_bins, from 2^24 products, numeric launches
    over several streams) -- webbase-like holds 256-thread block rows on both sides of the split;
    the split launches must run and the product equal the oracle's."""
    A = synth.SYNTH["webbase-1M"]()
    t2 = mhspgemm.Tool(tool.device)
    try:
        t = check(t2, A, A)
        assert t.flop >= 1 << 24
        assert t2.stat("multi_stream") == 1 and t2.stat("split") == 1, (t2.stat("split"), t.num_bins)
    finally:
        t2.close()
        A.d_release_csr()


@pytest.mark.parametrize("fork", ["0", "1"])
def test_near_groups_with_symbolic_fork(tool, fork, monkeypatch):
    """the rare symbolic bins on an aux stream (MHS_SYM_FORK=1) with near groups on:
    the near check then runs in launch_near after the aux stream's join -- verified groups and
    the oracle's C either way; the non-finite dissolve on the forked ordering too."""
    monkeypatch.setenv("MHS_SYM_FORK", fork)
    t2 = mhspgemm.Tool(tool.device)
    try:
        A = _perturbed_fem(7, 6, 24, 0.03, seed=31)
        t = check(t2, A, A)
        assert t.num_bins[6] + t.num_bins[7] > 0, t.num_bins
        assert t2.stat("near") == 1
        assert t2.stat("sym_fork") == (1 if fork == "1" else 0)
        v = A.val.copy()
        v[[5, 1000, 2500]] = np.inf
        v[4321] = np.nan
        An = mhspgemm.CSR(A.M, A.N, A.ptr, A.col, v)
        p, c, vv, _ = run_gpu(t2, An, An)
        Cp, Ci, Cv = orc.spgemm(An.ptr, An.col, An.val, An.ptr, An.col, An.val, An.N)
        assert np.array_equal(p, Cp) and np.array_equal(c, Ci)
        assert np.array_equal(np.isnan(vv), np.isnan(Cv)) and np.array_equal(np.isinf(vv), np.isinf(Cv))
        fin = np.isfinite(Cv)
        assert np.allclose(vv[fin], Cv[fin], rtol=RTOL, atol=ATOL)
    finally:
        t2.close()


@pytest.mark.parametrize("auto", ["12", "0"])
def test_numeric_first_without_probe(tool, auto, monkeypatch):
    """Round 5: short-row matrices below the probe's 512 K rows sort their tiny rows once, in
    symbolic, into value slots sized by the per-row bound (no hand-off); MHS_NFT_AUTO_AVG=0 keeps
    the two sorts.  Same C either way, on the tiny zoo and the short-row configs."""
    monkeypatch.setenv("MHS_NFT_AUTO_AVG", auto)
    t2 = mhspgemm.Tool(tool.device)
    try:
        (M, K, Ap, Ac, Av), (K2, N, Bp, Bc, Bv) = tiny_zoo(7)
        A = mhspgemm.CSR(M, K, Ap, Ac, Av)
        B = mhspgemm.CSR(K2, N, Bp, Bc, Bv)
        check(t2, A, B)
        for name in ("mac_econ_fwd500", "scircuit"):
            A = synth.SYNTH[name]()
            check(t2, A, A)
            A.d_release_csr()
        assert (t2.stat("nft") > 0) == (auto != "0"), t2.stat("nft")
    finally:
        t2.close()


@pytest.mark.parametrize("mode", ["nft", "plain", "notiny"])
def test_symbolic_scattered_sort_class(tool, mode, monkeypatch):
    """Round 5: rows of at most 512 products whose symbolic tables would not fit the small wave
    bin (a hub column's B row beside short ones; web-graph rows) count by a 64-lane register sort
    (symbolic bin 9) and k_scan sends them to numeric's 64-lane sort classes, since symbolic kept
    no masks for them -- with numeric-first slots (nft), without (plain), and off with the numeric
    tiny classes (notiny: those rows then count in tables and keep their masks)."""
    if mode == "plain":
        monkeypatch.setenv("MHS_NFT_AUTO_AVG", "0")
    if mode == "notiny":
        monkeypatch.setenv("MHS_NO_TINY_NUM", "1")
    t2 = mhspgemm.Tool(tool.device)
    try:
        for name in ("scircuit", "webbase-1M"):
            A = synth.SYNTH[name]()
            t = check(t2, A, A)
            if mode == "notiny":
                assert t.sym_bins[9] == 0, t.sym_bins
            else:
                # (scircuit-like's hub-column rows always need more than the small wave table;
                # which web-graph rows do depends on the symbolic table sizing)
                assert name != "scircuit" or t.sym_bins[9] > 0, t.sym_bins
                assert t.num_bins[12] + t.num_bins[13] >= t.sym_bins[9], t.num_bins
            A.d_release_csr()
    finally:
        t2.close()


# ---- round 6: launch plan speculation (MHS_OPT_SPECULATE, SpecArgs in mhs_internal.hpp) -------

def _host_c(C):
    try:
        return C.to_host()
    finally:
        C.release()


@pytest.mark.parametrize("nss", ["1", "4"])
@pytest.mark.parametrize("name", ["cant", "scircuit", "mac_econ_fwd500", "cop20k_A", "cant-perturbed"])
def test_speculated_plan_repeats(tool, name, nss, monkeypatch):
    """Calls after the first on the same operands queue the previous call's numeric plan behind
    k_scan; k_scan verifies it on the device.  Every call's C equals the oracle's, the second and
    later calls speculate and none misses -- synchronised, timed and unsynchronised calls alike.
    A plan dealt over several streams queues its call-stream launches ahead of the scan and the
    aux streams' after the hand-off (NumPhase); MHS_SPEC_NSS=1 keeps every launch on the call's
    stream -- both give the oracle's C."""
    from mhspgemm import _lib as L
    monkeypatch.setenv("MHS_SPEC_NSS", nss)
    A = synth.SYNTH[name]()
    A.H2D(tool.device)
    Cp, Ci, Cv = orc.spgemm(A.ptr, A.col, A.val, A.ptr, A.col, A.val, A.N)
    t2 = mhspgemm.Tool(tool.device)
    try:
        for it in range(4):
            if it == 3:
                t2.set_option(L.MHS_OPT_SYNC, 0)
            C, t = mhspgemm.spgemm(t2, A, A, timing=(it == 2))
            p, c, v = _host_c(C)
            assert np.array_equal(p, Cp) and np.array_equal(c, Ci), it
            assert mhspgemm.compare_tol(Cp, Ci, Cv, p, c, v, RTOL, ATOL)[0], it
        assert t2.stat("spec") == 3 and t2.stat("spec_miss") == 0, (t2.stat("spec"), t2.stat("spec_miss"))
    finally:
        t2.close()
        A.d_release_csr()


def test_speculated_plan_miss_and_values(tool, monkeypatch):
    """The same device arrays with new contents: a new pattern changes the Stats -- k_scan rejects
    the plan, its kernels return at once and the call reruns (MHS_STAT_SPEC_MISS); new values on
    the same pattern keep the plan (hit) and give the new values.  The rare bins the plan left
    out (empty in the first pattern) must run on the rerun."""
    import torch
    monkeypatch.setenv("MHS_SPEC_NSS", "4")  # (whatever streams the zoo's numeric phase takes)
    (M, K, Ap, Ac, Av), (K2, N, Bp, Bc, Bv) = bin_zoo()
    A = mhspgemm.CSR(M, K, Ap, Ac, Av)
    B = mhspgemm.CSR(K2, N, Bp, Bc, Bv)
    A.H2D(tool.device)
    B.H2D(tool.device)
    t2 = mhspgemm.Tool(tool.device)
    try:
        def run_and_check(Ah, Bh):
            C, _ = mhspgemm.spgemm(t2, A, B)
            p, c, v = _host_c(C)
            Cp, Ci, Cv = orc.spgemm(Ah[0], Ah[1], Ah[2], Bh[0], Bh[1], Bh[2], N)
            assert np.array_equal(p, Cp) and np.array_equal(c, Ci)
            assert mhspgemm.compare_tol(Cp, Ci, Cv, p, c, v, RTOL, ATOL)[0]

        run_and_check((Ap, Ac, Av), (Bp, Bc, Bv))
        run_and_check((Ap, Ac, Av), (Bp, Bc, Bv))
        assert t2.stat("spec") == 1 and t2.stat("spec_miss") == 0
        # values only: the plan holds
        Av2 = Av * 1.5 + 0.25
        A.d_val.copy_(torch.from_numpy(Av2))
        run_and_check((Ap, Ac, Av2), (Bp, Bc, Bv))
        assert t2.stat("spec") == 2 and t2.stat("spec_miss") == 0
        # a new pattern of A with the same nnz in the same arrays: rows' columns moved
        rng = np.random.default_rng(3)
        Ac2 = Ac.copy()
        for r in range(M):
            a0, a1 = int(Ap[r]), int(Ap[r + 1])
            if a1 > a0:
                Ac2[a0:a1] = np.sort(rng.choice(K, a1 - a0, replace=False)).astype(np.int32)
        A.d_col.copy_(torch.from_numpy(Ac2))
        run_and_check((Ap, Ac2, Av2), (Bp, Bc, Bv))
        assert t2.stat("spec") == 3 and t2.stat("spec_miss") == 1
        run_and_check((Ap, Ac2, Av2), (Bp, Bc, Bv))  # the rerun left its own plan: a hit
        assert t2.stat("spec") == 4 and t2.stat("spec_miss") == 1
        # the plan skipped empty rare symbolic bins somewhere in these calls, or it had none
        assert t2.stat("spec_skipped") >= 0
    finally:
        t2.close()


def test_speculated_plan_skips_empty_symbolic_launches(tool):
    """A matrix without rare symbolic rows: speculated calls leave out the empty k_sym_rare /
    k_sym_block<256> launches; a second matrix of the same sizes at the same addresses whose
    rows do need them is caught by the scan (its Stats differ) and reruns with them."""
    import torch
    A = synth.SYNTH["mac_econ_fwd500"]()
    A.H2D(tool.device)
    t2 = mhspgemm.Tool(tool.device)
    try:
        for _ in range(2):
            C, t = mhspgemm.spgemm(t2, A, A)
            C.release()
        assert t2.stat("spec") == 1 and t2.stat("spec_skipped") >= 1, (t2.stat("spec"), t2.stat("spec_skipped"))
        # one hub row: row 0 takes the columns of rows 1..k (same nnz: those rows give theirs up)
        p, c, v = A.ptr.copy(), A.col.copy(), A.val.copy()
        n0 = int(p[1] - p[0])
        hub = np.unique(np.concatenate([c[p[0]:p[1]], np.arange(0, A.N, max(1, A.N // 2000))]))[:2000]
        # rebuild a CSR with the same nnz: row 0 = hub, the last rows shortened to pay for it
        rows = [c[p[i]:p[i + 1]] for i in range(A.M)]
        extra = len(hub) - n0
        rows[0] = hub.astype(np.int32)
        i = A.M - 1
        while extra > 0:
            take = min(extra, len(rows[i]))
            rows[i] = rows[i][:len(rows[i]) - take]
            extra -= take
            i -= 1
        p2 = np.zeros(A.M + 1, np.int64)
        np.cumsum([len(r) for r in rows], out=p2[1:])
        c2 = np.concatenate(rows).astype(np.int32)
        assert len(c2) == A.nnz
        A.d_ptr.copy_(torch.from_numpy(p2.astype(np.int32)))
        A.d_col.copy_(torch.from_numpy(c2))
        C, t = mhspgemm.spgemm(t2, A, A)
        pp, cc, vv = _host_c(C)
        Cp, Ci, Cv = orc.spgemm(p2.astype(np.int32), c2, v, p2.astype(np.int32), c2, v, A.N)
        assert np.array_equal(pp, Cp) and np.array_equal(cc, Ci)
        assert mhspgemm.compare_tol(Cp, Ci, Cv, pp, cc, vv, RTOL, ATOL)[0]
        assert t2.stat("spec_miss") == 1
    finally:
        t2.close()
        A.d_release_csr()


@pytest.mark.parametrize("mode", ["default", "0"])
def test_speculated_calls_fork_rare_symbolic_rows(tool, mode, monkeypatch):
    """Speculated calls whose plan has rare symbolic rows (scircuit-like's k_sym_rare bins) run
    them on an aux stream beside k_sym_common (mhs_api.cpp, spec_fork_rare); MHS_SPEC_FORK=0 keeps
    them behind it.  Both give the oracle's C on every call."""
    if mode != "default":
        monkeypatch.setenv("MHS_SPEC_FORK", mode)
    A = synth.SYNTH["scircuit"]()
    A.H2D(tool.device)
    Cp, Ci, Cv = orc.spgemm(A.ptr, A.col, A.val, A.ptr, A.col, A.val, A.N)
    t2 = mhspgemm.Tool(tool.device)
    try:
        for it in range(3):
            C, _ = mhspgemm.spgemm(t2, A, A)
            p, c, v = _host_c(C)
            assert np.array_equal(p, Cp) and np.array_equal(c, Ci), it
            assert mhspgemm.compare_tol(Cp, Ci, Cv, p, c, v, RTOL, ATOL)[0], it
        assert t2.stat("spec") == 2 and t2.stat("spec_miss") == 0
        assert t2.stat("sym_fork") == (2 if mode == "default" else 0), t2.stat("sym_fork")
    finally:
        t2.close()
        A.d_release_csr()


def test_forked_speculated_plan_miss(tool):
    """A speculated call that forks its plan's rare symbolic rows, then the same arrays with a
    new pattern: k_scan rejects the plan and the call reruns without it -- the oracle's C on
    every call, the fork taken on the speculated ones."""
    import torch
    A = synth.SYNTH["scircuit"]()
    A.H2D(tool.device)
    t2 = mhspgemm.Tool(tool.device)
    try:
        def run_and_check(p_, c_, v_):
            C, _ = mhspgemm.spgemm(t2, A, A)
            pp, cc, vv = _host_c(C)
            Cp, Ci, Cv = orc.spgemm(p_, c_, v_, p_, c_, v_, A.N)
            assert np.array_equal(pp, Cp) and np.array_equal(cc, Ci)
            assert mhspgemm.compare_tol(Cp, Ci, Cv, pp, cc, vv, RTOL, ATOL)[0]

        run_and_check(A.ptr, A.col, A.val)
        run_and_check(A.ptr, A.col, A.val)
        assert t2.stat("spec") == 1 and t2.stat("sym_fork") == 1 and t2.stat("spec_miss") == 0
        rng = np.random.default_rng(11)
        c2 = A.col.copy()
        for r in range(0, A.M, 7):  # every 7th row's columns redrawn (same length, sorted)
            a0, a1 = int(A.ptr[r]), int(A.ptr[r + 1])
            if a1 > a0:
                c2[a0:a1] = np.sort(rng.choice(A.N, a1 - a0, replace=False)).astype(np.int32)
        A.d_col.copy_(torch.from_numpy(c2))
        run_and_check(A.ptr, c2, A.val)
        assert t2.stat("spec") == 2 and t2.stat("spec_miss") == 1, (t2.stat("spec"), t2.stat("spec_miss"))
        run_and_check(A.ptr, c2, A.val)  # the rerun's own plan: a hit
        assert t2.stat("spec_miss") == 1
    finally:
        t2.close()
        A.d_release_csr()


def test_speculation_off(tool):
    from mhspgemm import _lib as L
    A = synth.SYNTH["scircuit"]()
    A.H2D(tool.device)
    t2 = mhspgemm.Tool(tool.device)
    try:
        t2.set_option(L.MHS_OPT_SPECULATE, 0)
        for _ in range(3):
            C, _ = mhspgemm.spgemm(t2, A, A)
            C.release()
        assert t2.stat("spec") == 0
    finally:
        t2.close()
        A.d_release_csr()


def test_tiny_first_rows_negative_means_never(tool):
    """MHS_OPT_TINY_FIRST_ROWS < 0 turns numeric-first off, the probe-less mode below
    the threshold included (it had turned it on for every short-row matrix)."""
    from mhspgemm import _lib as L
    t2 = mhspgemm.Tool(tool.device)
    try:
        t2.set_option(L.MHS_OPT_TINY_FIRST_ROWS, -1)
        A = synth.SYNTH["mac_econ_fwd500"]()
        check(t2, A, A)
        assert t2.stat("nft") == 0
        A.d_release_csr()
    finally:
        t2.close()


def test_nft_slots_skipped_under_memory_budget(tool):
    """the probe-less numeric-first slots (M * 128 * 12 bytes) are left out when they do
    not fit the context's memory budget -- the call runs without them instead of chunking."""
    from mhspgemm import _lib as L
    A = synth.SYNTH["mac_econ_fwd500"]()  # slots 206 500 * 1536 B = 317 MB; workspace ~350 MB, C 59 MB
    t2 = mhspgemm.Tool(tool.device)
    try:
        t2.set_option(L.MHS_OPT_MEM_BUDGET, 520)
        check(t2, A, A)
        assert t2.stat("nft") == 0 and t2.chunked_calls() == 0
        A.d_release_csr()
    finally:
        t2.close()
