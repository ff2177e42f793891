"""The reference's own test suite (test/runtests.jl:23-190) restated over the GPU path:
six testsets x 200 sizes with the same generators (dense rand; test_matrix FE blocks) and the
same checks (lsolve!/rsolve! vs L\\b, U\\b; ldiv! vs A\\b before and after lu!).  Julia's
MersenneTwister(47) stream is not reproduced (numpy Generator seeded 47 instead).  The
reference compares UMFPACK with UMFPACK; against independent solvers the tolerance is
max(reference tol, 8 eps kappa(A)) (see ctol)."""
import glob
import os

import numpy as np
import pytest
import scipy.sparse as sp
import scipy.sparse.linalg as spla

import oracle as O
import smlu

pytestmark = pytest.mark.gpu

TOL = 1.0e-12
DENSE_TOL = 1.0e-10
NMAX = 200
HERE = os.path.dirname(os.path.abspath(__file__))


def isapprox(x, y, rtol, atol):
    return np.linalg.norm(x - y) <= max(atol, rtol * max(np.linalg.norm(x), np.linalg.norm(y)))


def ctol(A, tol):
    return max(tol, 8 * np.finfo(float).eps * np.linalg.cond(A.toarray()))


def test_reference_suite(gpu):
    rng = np.random.default_rng(47)
    fails = []
    # lsolve! dense (:38-53)
    for n in range(1, NMAX + 1):
        A = sp.csc_matrix(rng.random((n, n)))
        F = smlu.ParallelSparseLU(A)
        b = rng.random(n); x = b.copy()
        smlu.lsolve_(F, x)
        if not isapprox(x, spla.spsolve_triangular(F.L.tocsr(), b, lower=True), TOL, TOL):
            fails.append(("lsolve dense", n))
    # lsolve! sparse (:55-72)
    for nel in range(1, NMAX + 1):
        A = O.test_matrix(rng, nel, 5)
        F = smlu.ParallelSparseLU(A)
        n = A.shape[0]
        b = rng.random(n); x = b.copy()
        smlu.lsolve_(F, x)
        if not isapprox(x, spla.spsolve_triangular(F.L.tocsr(), b, lower=True), TOL, TOL):
            fails.append(("lsolve sparse", nel))
    # rsolve! dense (:74-88)
    for n in range(1, NMAX + 1):
        A = sp.csc_matrix(rng.random((n, n)))
        F = smlu.ParallelSparseLU(A)
        b = rng.random(n); x = b.copy()
        smlu.rsolve_(F, x)
        if not isapprox(x, spla.spsolve_triangular(F.U.tocsr(), b, lower=False), DENSE_TOL, DENSE_TOL):
            fails.append(("rsolve dense", n))
    # rsolve! sparse (:90-106)
    for nel in range(1, NMAX + 1):
        A = O.test_matrix(rng, nel, 5)
        F = smlu.ParallelSparseLU(A)
        n = A.shape[0]
        b = rng.random(n); x = b.copy()
        smlu.rsolve_(F, x)
        if not isapprox(x, spla.spsolve_triangular(F.U.tocsr(), b, lower=False), DENSE_TOL, DENSE_TOL):
            fails.append(("rsolve sparse", nel))
    # dense matrix (:108-146)
    for n in range(1, NMAX + 1):
        A = sp.csc_matrix(rng.random((n, n)))
        F = smlu.ParallelSparseLU(A)
        b = rng.random(n); x = np.empty(n)
        t = ctol(A, DENSE_TOL)
        smlu.ldiv_(x, F, b)
        ok = isapprox(x, np.linalg.solve(A.toarray(), b), t, t)
        b[:] = rng.random(n)
        smlu.ldiv_(x, F, b)
        ok &= isapprox(x, np.linalg.solve(A.toarray(), b), t, t)
        A = sp.csc_matrix(rng.random((n, n)))
        smlu.lu_(F, A)
        t = ctol(A, DENSE_TOL)
        b[:] = rng.random(n)
        smlu.ldiv_(x, F, b)
        ok &= isapprox(x, np.linalg.solve(A.toarray(), b), t, t)
        b[:] = rng.random(n)
        smlu.ldiv_(x, F, b)
        ok &= isapprox(x, np.linalg.solve(A.toarray(), b), t, t)
        if not ok:
            fails.append(("dense matrix", n))
    # sparse matrix (:148-188)
    for nel in range(1, NMAX + 1):
        A = O.test_matrix(rng, nel, 5)
        n = A.shape[0]
        F = smlu.ParallelSparseLU(A)
        b = rng.random(n); x = np.empty(n)
        t = ctol(A, TOL)
        smlu.ldiv_(x, F, b)
        ok = isapprox(x, spla.spsolve(A, b), t, t)
        b[:] = rng.random(n)
        smlu.ldiv_(x, F, b)
        ok &= isapprox(x, spla.spsolve(A, b), t, t)
        A = O.test_matrix(rng, nel, 5)
        smlu.lu_(F, A)
        t = ctol(A, TOL)
        b[:] = rng.random(n)
        smlu.ldiv_(x, F, b)
        ok &= isapprox(x, spla.spsolve(A, b), t, t)
        b[:] = rng.random(n)
        smlu.ldiv_(x, F, b)
        ok &= isapprox(x, spla.spsolve(A, b), t, t)
        if not ok:
            fails.append(("sparse matrix", nel))
    assert not fails, fails


GOLDEN = sorted(glob.glob(os.path.join(HERE, "golden", "*.npz")))


@pytest.mark.parametrize("path", GOLDEN, ids=[os.path.basename(p)[:-4] for p in GOLDEN])
def test_golden_with_given_pivots(gpu, path):
    """The committed fixtures' (p, q) handed over through smlu_create_with_pivots (the Julia
    shim's UMFPACK hand-over path): GPU factors and solution must match the fixture."""
    z = np.load(path, allow_pickle=False)
    n = int(z["n"])
    A = sp.csc_matrix((z["A_data"], z["A_indices"], z["A_indptr"]), shape=(n, n))
    L = sp.csc_matrix((z["L_data"], z["L_indices"], z["L_indptr"]), shape=(n, n))
    U = sp.csc_matrix((z["U_data"], z["U_indices"], z["U_indptr"]), shape=(n, n))
    # the whole §8(b) hand-over: (p, q) and the fixture's own L/U pattern
    F = smlu.ParallelSparseLU(A, p=z["p"], q=z["q"], L_pattern=L, U_pattern=U)
    assert F.stat("given_pattern") == 1 and F.stat("pattern_dropped") == 0
    assert np.array_equal(F.p, z["p"]) and np.array_equal(F.q, z["q"])
    assert np.array_equal(F.Rs, z["Rs"])
    for G, R in ((F.L, L), (F.U, U)):
        assert np.array_equal(G.indptr, R.indptr), "colptr differs from the fixture"
        assert np.array_equal(G.indices, R.indices), "rowval differs from the fixture"
        D = (G - R)
        assert abs(D).max() <= 1e-11 * max(1.0, abs(R).max())
    x = np.empty(n)
    smlu.ldiv_(x, F, z["b"])
    np.testing.assert_allclose(x, z["x"], rtol=1e-10, atol=1e-12)


def test_c1_fixture_default_analysis(gpu):
    """C1 (BASELINE configs[0]) through the default constructor: the GPU's own
    analysis and pivot choice reproduce the fixture's (p, q) bit for bit, its L/U pattern hashes,
    and its sampled values / column sums and solution to 1e-12."""
    from test_oracle import C1, check_c1_digest
    z = np.load(C1, allow_pickle=False)
    n = int(z["n"])
    A = sp.csc_matrix((z["A_data"], z["A_indices"], z["A_indptr"]), shape=(n, n))
    F = smlu.ParallelSparseLU(A)
    assert np.array_equal(F.q, z["q"]) and np.array_equal(F.p, z["p"])
    x = np.empty(n)
    smlu.ldiv_(x, F, z["b"])
    check_c1_digest(z, F.L, F.U, F.Rs, x, 1e-12)
    F.close()


def _pattern_case():
    z = np.load(os.path.join(HERE, "golden", "poisson2d_16.npz"), allow_pickle=False)
    n = int(z["n"])
    A = sp.csc_matrix((z["A_data"], z["A_indices"], z["A_indptr"]), shape=(n, n))
    L = sp.csc_matrix((z["L_data"], z["L_indices"], z["L_indptr"]), shape=(n, n))
    U = sp.csc_matrix((z["U_data"], z["U_indices"], z["U_indptr"]), shape=(n, n))
    return z, n, A, L, U


def test_given_pattern_with_dropped_fill(gpu):
    # UMFPACK leaves out fill entries that came out exactly zero: a given pattern that is a strict
    # subset of the structural fill is accepted, F.L / F.U come back on exactly that pattern with
    # the factor values at its positions, and pattern_dropped counts what it left out
    z, n, A, L, U = _pattern_case()
    keepL = np.ones(L.nnz, bool)
    Lc = L.tocoo()
    off = np.flatnonzero(Lc.row != Lc.col)
    keepL[off[::7]] = False          # every 7th strictly-lower entry of the fixture's L
    L2 = sp.csc_matrix((Lc.data[keepL], (Lc.row[keepL], Lc.col[keepL])), shape=(n, n))
    Uc = U.tocoo()
    keepU = np.ones(U.nnz, bool)
    offu = np.flatnonzero(Uc.row != Uc.col)
    keepU[offu[::5]] = False
    U2 = sp.csc_matrix((Uc.data[keepU], (Uc.row[keepU], Uc.col[keepU])), shape=(n, n))
    F = smlu.ParallelSparseLU(A, p=z["p"], q=z["q"], L_pattern=L2, U_pattern=U2)
    assert F.stat("pattern_dropped") == (L.nnz - L2.nnz) + (U.nnz - U2.nnz)
    for G, R, P in ((F.L, L, L2), (F.U, U, U2)):
        P = sp.csc_matrix(P)
        P.sort_indices()
        assert np.array_equal(G.indptr, P.indptr) and np.array_equal(G.indices, P.indices)
        # values at the kept positions are the factor's own
        Rk = R.multiply(P != 0).tocsc()
        Rk.sort_indices()
        assert abs(G - Rk).max() <= 1e-11 * max(1.0, abs(R).max())
    F.close()


def test_given_pattern_cleared_by_pattern_change(gpu):
    # lu!(F, A_new) with a new sparsity pattern re-analyses (src/SharedMemSparseLU.jl:252-273): the
    # handed-over UMFPACK pattern and (p, q) belong to the old A, so the new factors must come back
    # on their own structural fill, equal to the oracle's factorization of the new matrix
    from _parity import factor_parity
    z, n, A, L, U = _pattern_case()
    F = smlu.ParallelSparseLU(A, p=z["p"], q=z["q"], L_pattern=L, U_pattern=U)
    assert F.stat("given_pattern") == 1
    A2 = A.tolil()
    A2[0, n - 1] = -0.25          # one new off-diagonal pair: a different pattern and new fill
    A2[n - 1, 0] = -0.25
    A2 = sp.csc_matrix(A2)
    A2.sort_indices()
    smlu.lu_(F, A2)
    assert F.stat("given_pattern") == 0 and F.stat("pattern_dropped") == 0
    factor_parity(A2, F)
    b = np.random.default_rng(9).random(n)
    x = np.empty(n)
    smlu.ldiv_(x, F, b)
    assert np.abs(A2 @ x - b).max() <= 1e-12 * np.abs(b).max() * 10
    F.close()


@pytest.mark.parametrize("bad", ["outside_fill", "no_diagonal", "upper_in_L"])
def test_given_pattern_rejected(gpu, bad):
    z, n, A, L, U = _pattern_case()
    L2 = L.tolil()
    if bad == "outside_fill":
        # an entry the structural fill of (Rs.*A)[p, q] does not have
        Ld = L.toarray() != 0
        i, j = np.argwhere(~Ld & np.tri(n, k=-1, dtype=bool))[0]
        L2[i, j] = 1.0
    elif bad == "no_diagonal":
        L2[3, 3] = 0.0
    else:
        L2[0, 5] = 1.0
    L2 = sp.csc_matrix(L2)
    L2.eliminate_zeros()
    with pytest.raises(smlu.SmluError) as ei:
        smlu.ParallelSparseLU(A, p=z["p"], q=z["q"], L_pattern=L2, U_pattern=U)
    assert "(-2)" in str(ei.value)
