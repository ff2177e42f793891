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
    F = smlu.ParallelSparseLU(A, p=z["p"], q=z["q"])
    assert np.array_equal(F.p, z["p"]) and np.array_equal(F.q, z["q"])
    assert np.array_equal(F.Rs, z["Rs"])
    L = sp.csc_matrix((z["L_data"], z["L_indices"], z["L_indptr"]), shape=(n, n))
    U = sp.csc_matrix((z["U_data"], z["U_indices"], z["U_indptr"]), shape=(n, n))
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
