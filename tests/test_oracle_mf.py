"""CPU tests of the multifrontal pivot-rule oracle (oracle/mf.c), the independent restatement the
GPU's pivot decisions are checked against (tests/_parity.py: pivot_parity).

Pinned against LAPACK: with the diagonal preference switched off (diag_tol = 1: keep a_kk only if
it is a largest candidate) and one front holding every row, the rule is plain partial pivoting,
and the oracle's row order must equal dgetrf's (scipy.linalg.lu_factor, first maximum on ties)
bit for bit.  Then the threshold rule (diag_tol = 0.1, UMFPACK's default pivot tolerance), the
64 x 64 tile candidate sets, the re-pivoting decision and OpenMP determinism on real assembly
trees from the host plan."""
import numpy as np
import pytest
import scipy.linalg as sla
import scipy.sparse as sp

import oracle as O
from smlu import matrices as mats
from smlu.plan import Plan


def one_front(n):
    return dict(first=np.array([0, n]), parent=np.array([-1]), rowptr=np.array([0, 0]),
                rows=np.zeros(0, np.int64), p0=np.arange(n))


def lapack_perm(B):
    """Row order of dgetrf(B): perm[k] = original row in position k."""
    _, piv = sla.lu_factor(B)
    perm = np.arange(B.shape[0])
    for k, pk in enumerate(piv):
        perm[[k, pk]] = perm[[pk, k]]
    return perm


@pytest.mark.parametrize("n", [1, 2, 5, 33, 64, 65, 130, 200])
def test_partial_pivoting_equals_lapack(n):
    rng = np.random.default_rng(n)
    D = rng.random((n, n)) - 0.5
    A = sp.csc_matrix(D)
    Rs = O.rowscale(A)
    mf = O.MultifrontalOracle(A, np.arange(n), one_front(n), [1], diag_tol=1.0)
    assert mf.factor(A.data) == 0
    assert np.array_equal(mf.Rs, Rs)
    assert np.array_equal(mf.p, lapack_perm(Rs[:, None] * D))
    mf.close()


def test_threshold_rule_keeps_diagonal_within_tolerance():
    # diag_tol 0.1: the diagonal stays unless another candidate is 10x larger; every chosen pivot
    # satisfies |u_kk| >= 0.1 max|candidates|, i.e. every multiplier of L is at most 10
    n = 150
    rng = np.random.default_rng(3)
    D = rng.random((n, n)) + np.diag(rng.random(n) * 0.3)
    A = sp.csc_matrix(D)
    mf = O.MultifrontalOracle(A, np.arange(n), one_front(n), [1], diag_tol=0.1)
    assert mf.factor(A.data) == 0
    p = mf.p
    ref = O.OracleLU(A, p, np.arange(n))
    assert abs(ref.L).max() <= 10.0 * (1 + 1e-12)
    assert not np.array_equal(p, lapack_perm(mf.Rs[:, None] * D))   # the preference matters
    assert (p == np.arange(n)).sum() > 0.2 * n                        # many diagonals kept
    mf.close()


def test_tile_candidates_stay_in_their_tile():
    # mode 2: only rows of the 64 x 64 diagonal tile are candidates
    n = 200
    rng = np.random.default_rng(4)
    D = rng.random((n, n))
    A = sp.csc_matrix(D)
    mf = O.MultifrontalOracle(A, np.arange(n), one_front(n), [2], diag_tol=0.1)
    mf.factor(A.data)
    p = mf.p
    assert not np.array_equal(p, np.arange(n))
    assert np.array_equal(p // 64, np.arange(n) // 64)
    # the same matrix in mode 1 picks rows across tiles
    mf1 = O.MultifrontalOracle(A, np.arange(n), one_front(n), [1], diag_tol=0.1)
    mf1.factor(A.data)
    assert not np.array_equal(mf1.p // 64, np.arange(n) // 64)
    # tile pivoting on this matrix accepts weak pivots (rows outside the tile dominate): flagged
    assert mf.flags[0] & 2
    mf.close()
    mf1.close()


def test_singular_column_flagged():
    n = 70
    D = np.random.default_rng(5).random((n, n))
    D[:, 10] = 0.0
    A = sp.csc_matrix(D)
    A.eliminate_zeros()
    A = sp.csc_matrix(A)
    mf = O.MultifrontalOracle(A, np.arange(n), one_front(n), [1])
    assert mf.factor(A.data) == 1 and mf.flags[0] & 1
    mf.close()


def _tree(A, **kw):
    P = Plan(A, **kw)
    first, parent, rowptr, rows, p0 = P.fronts()
    return P.q(), dict(first=first, parent=parent, rowptr=rowptr, rows=rows, p0=p0)


@pytest.mark.parametrize("case", ["poisson3d", "fe", "random"])
def test_multifrontal_factor_on_plan_tree(case):
    # real assembly trees: the oracle's pivots give an exact LU of (Rs.*A)[p, q] (fixed-pivot
    # oracle with that p) and dominant matrices keep the diagonal everywhere
    if case == "poisson3d":
        A = mats.poisson3d(9)
    elif case == "fe":
        A = O.test_matrix(np.random.default_rng(7), 60)
    else:
        A = sp.csc_matrix(mats.random_dominant(600, 0.01, seed=3))
    A = sp.csc_matrix(A)
    A.sort_indices()
    q, fr = _tree(A)
    modes = O.front_modes(fr, 0, O.dominant(A))
    # fe: diag_tol 0.1 so that rows are exchanged (UMFPACK's 0.001 keeps this FE matrix's diagonal)
    mf = O.MultifrontalOracle(A, q, fr, modes, diag_tol=0.1 if case == "fe" else 0.001)
    assert mf.factor(A.data) == 0
    p = mf.p
    assert np.array_equal(np.sort(p), np.arange(A.shape[0]))
    if case != "fe":
        assert np.array_equal(p, q)
    else:
        assert not np.array_equal(p, q)
    ref = O.OracleLU(A, p, q)
    B = (sp.diags(ref.Rs) @ A).tocsr()[p][:, q]
    assert abs(ref.L @ ref.U - B).max() <= 1e-12 * abs(B).max()
    mf.close()


def test_threads_are_bitwise_deterministic():
    # OpenMP over fronts and inside large fronts does not change any pivot (every entry sees the
    # same operations in the same order)
    A = sp.csc_matrix(O.test_matrix(np.random.default_rng(8), 150))
    A.sort_indices()
    q, fr = _tree(A)
    ps = []
    for t in (1, 4):
        mf = O.MultifrontalOracle(A, q, fr, None, threads=t)
        mf.factor(A.data)
        ps.append(mf.p)
        mf.close()
    assert np.array_equal(ps[0], ps[1])


def test_repivot_restatement():
    # a front with weak diagonal-tile pivots: the restated GPU decision re-factors with full
    # candidates (pivmode 1), after which no front is weak
    rng = np.random.default_rng(21)
    n = 700
    D = rng.random((n, n))
    for b0 in range(0, n, 64):
        b1 = min(n, b0 + 64)
        D[b0:b1, b0:b1] = 1e-2 * rng.random((b1 - b0, b1 - b0)) + 1e-2 * np.eye(b1 - b0)
    A = sp.csc_matrix(D)
    q, fr = _tree(A)
    p, pm, modes, flags = O.gpu_pivot_choice(A, q, fr)
    assert pm == 1 and (modes != 2).all() and not (flags & 2).any()
    # dominant values never re-pivot and keep the diagonal
    D2 = D + np.diag(D.sum(axis=1) + 1)
    p2, pm2, modes2, _ = O.gpu_pivot_choice(sp.csc_matrix(D2), q, fr)
    assert pm2 == 0 and (modes2 == 2).any() and np.array_equal(p2, q)


def fold_complex(L, U, p, q, n):
    """Python restatement of complex.cpp: export_complex -- the complex n x n factors from the scalar
    LU of the real-equivalent K under pair-preserving pivots, pairs kept in either order."""
    sw = p[0::2] > p[1::2]
    pc, qc = np.minimum(p[0::2], p[1::2]) // 2, q[0::2] // 2
    nsign = np.ones(2 * n)
    nsign[1::2][sw] = -1.0
    Ld, Ud = L.toarray(), U.toarray()
    Lr = nsign[:, None] * Ld * nsign[None, :]          # N L N
    Lc = Lr[1::2, 1::2] - 1j * Lr[0::2, 1::2]           # real: row 2i+1, imag: -row 2i (odd columns)
    Uc = Ud[0::2, 0::2] - 1j * Ud[0::2, 1::2]           # even rows of columns 2j, 2j+1
    d = np.where(sw, -1j, 1.0)
    return (Lc * d[None, :] / d[:, None]), Uc / d[:, None], pc, qc


@pytest.mark.parametrize("case", ["imaginary_diagonal", "random", "fe"])
def test_pair_rule_keeps_complex_pairs(case):
    # ComplexF64 handles pivot the real-equivalent K pair by pair (mf.c: factor_front, pairs):
    # the row order keeps every (2i, 2i+1) pair adjacent, and the folded complex factors satisfy
    # L U == (Rs.*A)[p, q] with L unit lower (a swap inside a pair folds back as a row rotation)
    rng = np.random.default_rng(3)
    n = 40
    if case == "imaginary_diagonal":
        A = sp.random(n, n, density=0.15, random_state=np.random.RandomState(1), format="csc") * (1 + 0.5j)
        A = sp.csc_matrix(A + sp.diags(1j * (3 + rng.random(n))))
    elif case == "random":
        D = rng.random((n, n)) + 1j * rng.random((n, n))
        A = sp.csc_matrix(D)
    else:
        F = O.test_matrix(np.random.default_rng(47), 9)
        A = sp.csc_matrix(F + 1j * (F != 0).multiply(np.random.default_rng(5).random(F.shape)))
    n = A.shape[0]
    K = O.real_equivalent(A)
    m = K.shape[0]
    q = np.arange(m)
    mf = O.MultifrontalOracle(K, q, one_front(m), [1], pairs=True)
    assert mf.factor(K.data) == 0
    p = mf.p
    mf.close()
    assert np.array_equal(np.sort(np.minimum(p[0::2], p[1::2]) // 2), np.arange(n))
    assert np.all(np.abs(p[0::2] - p[1::2]) == 1) and np.all(np.minimum(p[0::2], p[1::2]) % 2 == 0)
    if case == "imaginary_diagonal":
        assert (p[0::2] > p[1::2]).any()    # some pairs were swapped inside
    ref = O.OracleLU(K, p, q)
    Lc, Uc, pc, qc = fold_complex(ref.L, ref.U, p, q, n)
    Rs = ref.Rs[0::2]   # rows 2i, 2i+1 sum the same magnitudes (in another order: equal to rounding)
    B = (sp.diags(Rs) @ A).toarray()[pc][:, qc]
    assert np.allclose(np.diag(Lc), 1.0) and np.allclose(np.triu(Lc, 1), 0) and np.allclose(np.tril(Uc, -1), 0)
    assert np.abs(Lc @ Uc - B).max() <= 1e-12 * np.abs(B).max()
