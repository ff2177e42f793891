"""CPU tests of the oracle (test infrastructure): golden fixtures, UMFPACK contract, LAPACK
known answers, the reference's chunked-solve layout, and the reference's own six testsets
(test/runtests.jl:38-188) restated with the oracle as the factorization."""
import glob
import os
import sys

import numpy as np
import pytest
import scipy.linalg as sla
import scipy.sparse as sp
import scipy.sparse.linalg as spla

import oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
TOL = 1.0e-12        # test/runtests.jl:25
DENSE_TOL = 1.0e-10  # test/runtests.jl:26


def isapprox(x, y, rtol, atol):
    return np.linalg.norm(x - y) <= max(atol, rtol * max(np.linalg.norm(x), np.linalg.norm(y)))


def ctol(A, tol):
    """The reference compares UMFPACK against UMFPACK (A \\ b), so its fixed 1e-12/1e-10 hold
    even for ill-conditioned random inputs.  Against an independent solver the achievable
    agreement is ~kappa(A)*eps: tolerance = max(reference tol, 8*eps*kappa(A))."""
    k = np.linalg.cond(A.toarray() if sp.issparse(A) else A)
    return max(tol, 8 * np.finfo(float).eps * k)


def load(path):
    z = np.load(path, allow_pickle=False)
    n = int(z["n"])
    A = sp.csc_matrix((z["A_data"], z["A_indices"], z["A_indptr"]), shape=(n, n))
    L = sp.csc_matrix((z["L_data"], z["L_indices"], z["L_indptr"]), shape=(n, n))
    U = sp.csc_matrix((z["U_data"], z["U_indices"], z["U_indptr"]), shape=(n, n))
    return A, z, L, U


GOLDEN = sorted(glob.glob(os.path.join(HERE, "golden", "*.npz")))


def test_golden_present():
    assert len(GOLDEN) >= 10


@pytest.mark.parametrize("path", GOLDEN, ids=[os.path.basename(p)[:-4] for p in GOLDEN])
def test_oracle_matches_golden(path):
    A, z, L, U = load(path)
    F = O.OracleLU(A, z["p"], z["q"])
    assert np.array_equal(F.Rs, z["Rs"])
    for G, R in ((F.L, L), (F.U, U)):
        assert np.array_equal(G.indptr, R.indptr) and np.array_equal(G.indices, R.indices)
        np.testing.assert_allclose(G.data, R.data, rtol=1e-14, atol=1e-15)
    x = np.empty(A.shape[0])
    F.ldiv(x, z["b"])
    np.testing.assert_allclose(x, z["x"], rtol=1e-13, atol=1e-14)


C1 = os.path.join(HERE, "golden", "c1", "c1_random_1000.npz")


def check_c1_digest(z, L, U, Rs, x, rtol):
    """The C1 fixture's digests (tests/golden/make_golden.py: save_c1) against factors L, U."""
    sys.path.insert(0, os.path.join(HERE, "golden"))
    from make_golden import factor_digest, pattern_hash
    assert np.array_equal(Rs, z["Rs"]), "row scaling must be bitwise identical"
    for tag, M in (("L", L), ("U", U)):
        assert M.nnz == int(z[f"{tag}_nnz"]) and pattern_hash(M) == str(z[f"{tag}_hash"]), f"{tag} pattern differs"
        cs, sq, vals = factor_digest(M, z[f"{tag}_pick"])
        np.testing.assert_allclose(vals, z[f"{tag}_pickval"], rtol=rtol, atol=rtol)
        np.testing.assert_allclose(cs, z[f"{tag}_colsum"], rtol=rtol, atol=rtol * np.abs(z[f"{tag}_colsum"]).max())
        np.testing.assert_allclose(sq, z[f"{tag}_colsq"], rtol=rtol, atol=rtol * np.abs(z[f"{tag}_colsq"]).max())
    np.testing.assert_allclose(x, z["x"], rtol=rtol, atol=rtol)


def test_c1_fixture_oracle_and_plan():
    """C1 (n=1000, seed 47).  The generator is deterministic: the matrix, the
    plan's default column order and the oracle's factors reproduce the committed digests."""
    from smlu import matrices as mats
    from smlu.plan import Plan
    z = np.load(C1, allow_pickle=False)
    n = int(z["n"])
    A = sp.csc_matrix((z["A_data"], z["A_indices"], z["A_indptr"]), shape=(n, n))
    A0 = mats.random_dominant(1000, 0.01, 47)
    assert np.array_equal(A0.indptr, A.indptr) and np.array_equal(A0.indices, A.indices)
    assert np.array_equal(A0.data, A.data)
    assert np.array_equal(Plan(A).q(), z["q"]), "the analysis' column order changed"
    F = O.OracleLU(A, z["p"], z["q"])
    x = np.empty(n)
    F.ldiv(x, z["b"])
    check_c1_digest(z, F.L, F.U, F.Rs, x, 1e-14)


def _rand_sparse(rng, n, dens):
    A = sp.random(n, n, density=dens, random_state=rng, format="csc") + sp.diags(1.0 + rng.random(n))
    return sp.csc_matrix(A)


@pytest.mark.parametrize("seed", range(6))
def test_contract_L_times_U(seed):
    """F.L*F.U == (F.Rs .* A)[F.p, F.q]  (src/SharedMemSparseLU.jl:305-316)."""
    rng = np.random.default_rng(seed)
    A = _rand_sparse(rng, 60, 0.05)
    lu = spla.splu(A, permc_spec="COLAMD", diag_pivot_thresh=0.1)
    p = lu.perm_r.argsort()  # SuperLU orders as "new -> old": L*U == A[p][:, q]
    q = lu.perm_c.argsort()
    F = O.OracleLU(A, p, q)
    B = (sp.diags(F.Rs) @ A).tocsr()[p][:, q]
    assert abs(F.L @ F.U - B).max() <= 1e-12 * abs(B).max()
    # L: unit diagonal stored first, rows sorted; U: diagonal last
    for j in range(A.shape[0]):
        s, e = F.L.indptr[j], F.L.indptr[j + 1]
        assert F.L.indices[s] == j and F.L.data[s] == 1.0
        assert np.all(np.diff(F.L.indices[s:e]) > 0)
        s, e = F.U.indptr[j], F.U.indptr[j + 1]
        assert F.U.indices[e - 1] == j


@pytest.mark.parametrize("n", [1, 4, 9, 31])
def test_lapack_known_answer(n):
    """With LAPACK's own row order the fixed-pivot oracle reproduces dgetrf's L and U."""
    rng = np.random.default_rng(n)
    A = sp.csc_matrix(rng.random((n, n)))
    Rs = O.rowscale(A)
    P, _, _ = sla.lu((sp.diags(Rs) @ A).toarray())
    p = np.argmax(P, axis=0)
    F = O.OracleLU(A, p, np.arange(n), Rs)
    _, Ls, Us = sla.lu((sp.diags(Rs) @ A).toarray()[p])
    np.testing.assert_allclose(F.L.toarray(), Ls, rtol=1e-12, atol=1e-13)
    np.testing.assert_allclose(F.U.toarray(), Us, rtol=1e-12, atol=1e-13)


def test_rowscale_zero_row():
    A = sp.csc_matrix(np.array([[2.0, -1.0], [0.0, 0.0]]))
    np.testing.assert_array_equal(O.rowscale(A), [1 / 3, 1.0])


@pytest.mark.parametrize("cs", [None, 1, 3, 8, 1000])
def test_chunked_solve_restatement(cs):
    """Reference chunk layout (get_chunking_parameters/fill_chunks!/lsolve!/rsolve!, incl. the
    negated rectangles and the back-to-front U chunks) == plain CSC triangular solves."""
    rng = np.random.default_rng(7)
    A = O.test_matrix(rng, 9, 5)
    lu = spla.splu(A, permc_spec="NATURAL", diag_pivot_thresh=1.0)
    F = O.OracleLU(A, lu.perm_r.argsort(), np.arange(A.shape[0]))
    C = O.ChunkedSolve(F.L, F.U, cs)
    b = rng.random(A.shape[0])
    np.testing.assert_allclose(C.lsolve(b.copy()), F.lsolve(b.copy()), rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(C.rsolve(b.copy()), F.rsolve(b.copy()), rtol=1e-10, atol=1e-10)


def test_chunk_geometry_quirks():
    """Q1: chunk_size clamped to n; Q2: U chunks generated from the back; Q3: negated rects."""
    L = sp.csc_matrix(np.tril(np.ones((5, 5))))
    U = sp.csc_matrix(np.triu(np.ones((5, 5))))
    C = O.ChunkedSolve(L, U, 8)
    assert C.chunk_size == 5 and C.total_chunks == 1
    C = O.ChunkedSolve(L, U, 2)
    assert C.total_chunks == 3
    assert C.ucols[0] == (5, 5) and C.ucols[-1] == (1, 2)   # last partial chunk first (Q2)
    assert C.lrows[0] == (3, 5)
    assert np.all(C.Lchunks[1] == -1.0)                    # rectangle holds -L (Q3)


# ---- the reference's six testsets (test/runtests.jl:38-188), oracle as the factorization ----
def _pivots(A):
    """A stable pivot sequence for the fixed-pivot oracle: SuperLU partial pivoting."""
    lu = spla.splu(sp.csc_matrix(A), permc_spec="COLAMD", diag_pivot_thresh=1.0)
    return lu.perm_r.argsort(), lu.perm_c.argsort()


NS = list(range(1, 41)) + [57, 100, 151, 200]


@pytest.mark.parametrize("n", NS)
def test_reference_suite_dense(n):
    rng = np.random.default_rng(1000 + n)
    A = sp.csc_matrix(rng.random((n, n)))
    F = O.OracleLU(A, *_pivots(A))
    b = rng.random(n)
    x = F.lsolve(b.copy())                              # lsolve! dense (:38-53)
    assert isapprox(x, spla.spsolve_triangular(F.L.tocsr(), b, lower=True), TOL, TOL)
    x = F.rsolve(b.copy())                              # rsolve! dense (:74-88)
    assert isapprox(x, spla.spsolve_triangular(F.U.tocsr(), b, lower=False), DENSE_TOL, DENSE_TOL)
    x = np.empty(n)                                      # dense matrix (:108-146)
    F.ldiv(x, b)
    t = ctol(A, DENSE_TOL)
    assert isapprox(x, np.linalg.solve(A.toarray(), b), t, t)
    A2 = sp.csc_matrix(rng.random((n, n)))               # lu! with new values (:129-131)
    F = O.OracleLU(A2, *_pivots(A2))
    b = rng.random(n)
    F.ldiv(x, b)
    t = ctol(A2, DENSE_TOL)
    assert isapprox(x, np.linalg.solve(A2.toarray(), b), t, t)


@pytest.mark.parametrize("nel", NS)
def test_reference_suite_sparse(nel):
    rng = np.random.default_rng(2000 + nel)
    A = O.test_matrix(rng, nel, 5)
    n = A.shape[0]
    F = O.OracleLU(A, *_pivots(A))
    b = rng.random(n)
    x = F.lsolve(b.copy())                              # lsolve! sparse (:55-72)
    assert isapprox(x, spla.spsolve_triangular(F.L.tocsr(), b, lower=True), TOL, TOL)
    x = F.rsolve(b.copy())                              # rsolve! sparse (:90-106)
    assert isapprox(x, spla.spsolve_triangular(F.U.tocsr(), b, lower=False), DENSE_TOL, DENSE_TOL)
    x = np.empty(n)                                      # sparse matrix (:148-188)
    F.ldiv(x, b)
    t = ctol(A, TOL)
    assert isapprox(x, spla.spsolve(A, b), t, t)
    A2 = O.test_matrix(rng, nel, 5)                      # lu! same pattern new values (:172-173)
    F = O.OracleLU(A2, *_pivots(A2))
    b = rng.random(n)
    F.ldiv(x, b)
    t = ctol(A2, TOL)
    assert isapprox(x, spla.spsolve(A2, b), t, t)


def complex_fe(rng, nel, ngr=5):
    """The reference's FE fixture (test/runtests.jl:12-21) with complex values on its pattern."""
    A = O.test_matrix(rng, nel, ngr).tocsc()
    A.sort_indices()
    Z = A.astype(np.complex128)
    Z.data = Z.data + 1j * (rng.random(A.nnz) - 0.5)
    return Z


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_real_equivalent_embedding(seed):
    """K (oracle.real_equivalent) acts on interleaved vectors exactly as A on complex ones."""
    rng = np.random.default_rng(seed)
    A = complex_fe(rng, 7)
    n = A.shape[0]
    K = O.real_equivalent(A)
    assert K.shape == (2 * n, 2 * n) and K.nnz == 4 * A.nnz and K.has_sorted_indices
    x = rng.random(n) + 1j * rng.random(n)
    assert np.allclose(K @ x.view(np.float64), (A @ x).view(np.float64), rtol=0, atol=1e-14)


@pytest.mark.parametrize("nel", [1, 4, 12])
def test_oracle_complex_solve_vs_superlu(nel):
    """The oracle's LU of K with a pairwise column order solves the complex system: pinned
    against scipy's complex SuperLU at the reference's sparse tolerance (1e-12)."""
    rng = np.random.default_rng(100 + nel)
    A = complex_fe(rng, nel)
    n = A.shape[0]
    K = O.real_equivalent(A)
    order = np.argsort(rng.random(n))            # any complex order, expanded to pairs
    q = np.empty(2 * n, np.int64)
    q[0::2], q[1::2] = 2 * order, 2 * order + 1
    Rs = O.rowscale(K)
    assert np.allclose(Rs[0::2], Rs[1::2], rtol=1e-15, atol=0)   # SUM scaling: |x| + |y| per entry
    ref = O.OracleLU(K, q, q, Rs)
    assert ref.status == 0
    b = rng.random(n) + 1j * rng.random(n)
    xr = np.empty(2 * n)
    ref.ldiv(xr, b.view(np.float64).copy())
    x = xr.view(np.complex128)
    xs = spla.spsolve(A.tocsc(), b)
    assert np.linalg.norm(x - xs) <= 1e-12 * max(np.linalg.norm(x), 1.0) * max(1.0, np.linalg.cond(A.toarray()) / 1e3)
