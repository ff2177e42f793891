"""GPU parity tests: libsmlu.so (HIP, gfx950) against the CPU oracle (oracle/) and against
independent solvers, at the reference's tolerances (test/runtests.jl:25-26)."""
import numpy as np
import pytest
import scipy.linalg as sla
import scipy.sparse as sp
import scipy.sparse.linalg as spla

import oracle as O
import smlu
from smlu import matrices as mats

pytestmark = pytest.mark.gpu

from _parity import DENSE_TOL, TOL, assert_same_pattern, factor_parity, isapprox, tile_pivoting_matrix  # noqa: F401


@pytest.mark.parametrize("N", [4, 10, 23])
def test_poisson2d_factors_identical_pattern(gpu, N):
    A = mats.poisson2d(N)
    F = smlu.ParallelSparseLU(A)
    factor_parity(A, F)
    # diagonally dominant M-matrix: pivot order = column order (no swaps)
    assert np.array_equal(F.p, F.q)
    Lpat = smlu.Plan(A).L_pattern()
    G = F.L.copy(); G.data[:] = 1
    assert abs(G - Lpat).count_nonzero() == 0


@pytest.mark.parametrize("N,grid", [(6, True), (9, False), (13, True)])
def test_poisson3d_factors(gpu, N, grid):
    A = mats.poisson3d(N)
    F = smlu.ParallelSparseLU(A, grid=(N, N, N) if grid else None)
    factor_parity(A, F)
    assert np.array_equal(F.p, F.q)
    b = np.random.default_rng(1).random(A.shape[0])
    x = np.empty_like(b)
    smlu.ldiv_(x, F, b)
    assert isapprox(x, spla.spsolve(A, b), TOL, TOL)


@pytest.mark.parametrize("make", [lambda: mats.poisson2d(30), lambda: mats.poisson3d(12),
                                  lambda: O.test_matrix(np.random.default_rng(3), 57, 5)],
                         ids=["poisson2d_30", "poisson3d_12", "fe_57"])
def test_amd_ordering_factors(gpu, make):
    # SMLU_ORDER_AMD: factors against the oracle on the same (p, q), solve against SuperLU
    A = sp.csc_matrix(make())
    F = smlu.ParallelSparseLU(A, ordering="amd")
    factor_parity(A, F, rtol=1e-10)
    assert F.stat("nnzLU") > 0
    b = np.random.default_rng(2).random(A.shape[0])
    x = np.empty_like(b)
    smlu.ldiv_(x, F, b)
    assert isapprox(x, spla.spsolve(A, b), TOL, TOL)


@pytest.mark.parametrize("nel", [1, 2, 3, 7, 20, 57, 200])
def test_fe_matrix_ldiv(gpu, nel):
    rng = np.random.default_rng(47 + nel)
    A = O.test_matrix(rng, nel, 5)
    n = A.shape[0]
    F = smlu.ParallelSparseLU(A)
    factor_parity(A, F, rtol=1e-10)
    b = rng.random(n)
    x = np.empty(n)
    smlu.ldiv_(x, F, b)
    assert isapprox(x, spla.spsolve(A, b), TOL, TOL)


@pytest.mark.parametrize("n", [1, 2, 5, 17, 64, 130, 200, 333])
def test_dense_ldiv_and_refactor(gpu, n):
    rng = np.random.default_rng(n)
    A = sp.csc_matrix(rng.random((n, n)))
    F = smlu.ParallelSparseLU(A)
    b = rng.random(n)
    x = np.empty(n)
    smlu.ldiv_(x, F, b)
    assert isapprox(x, np.linalg.solve(A.toarray(), b), DENSE_TOL, DENSE_TOL)
    A2 = sp.csc_matrix(rng.random((n, n)))
    smlu.lu_(F, A2)
    b = rng.random(n)
    smlu.ldiv_(x, F, b)
    assert isapprox(x, np.linalg.solve(A2.toarray(), b), DENSE_TOL, DENSE_TOL)


def test_lsolve_rsolve(gpu):
    rng = np.random.default_rng(3)
    A = O.test_matrix(rng, 30, 5)
    F = smlu.ParallelSparseLU(A)
    n = A.shape[0]
    b = rng.random(n)
    x = b.copy()
    smlu.lsolve_(F, x)
    assert isapprox(x, spla.spsolve_triangular(F.L.tocsr(), b, lower=True), TOL, TOL)
    x = b.copy()
    smlu.rsolve_(F, x)
    assert isapprox(x, spla.spsolve_triangular(F.U.tocsr(), b, lower=False), DENSE_TOL, DENSE_TOL)


def test_random_dominant_c1(gpu):
    A = mats.random_dominant(1000, 0.01, 47)
    F = smlu.ParallelSparseLU(A)
    factor_parity(A, F, rtol=1e-11)
    b = np.random.default_rng(2).random(1000)
    x = np.empty(1000)
    smlu.ldiv_(x, F, b)
    assert isapprox(x, spla.spsolve(A, b), TOL, TOL)


def test_blocked_tile_mode_dominant(gpu):
    # ns > 512 -> diagonal-tile pivoting path (mode 2) on a dense dominant matrix
    n = 700
    rng = np.random.default_rng(5)
    D = rng.random((n, n))
    D += np.diag(D.sum(axis=1) + 1)
    A = sp.csc_matrix(D)
    F = smlu.ParallelSparseLU(A)
    b = rng.random(n)
    x = np.empty(n)
    smlu.ldiv_(x, F, b)
    assert isapprox(x, np.linalg.solve(D, b), DENSE_TOL, DENSE_TOL)
    factor_parity(A, F, rtol=1e-11)


def _tile_pivoting_matrix(n, seed):
    return tile_pivoting_matrix(n, seed)


@pytest.mark.parametrize("n", [700, 1100])
def test_blocked_tile_mode_pivoting(gpu, n):
    # diagonal-tile pivoting with real row exchanges (k_panel_tile64); parity with the oracle run
    # on the GPU's own final (p, q) and a solve against LAPACK
    D = _tile_pivoting_matrix(n, 11 + n)
    A = sp.csc_matrix(D)
    F = smlu.ParallelSparseLU(A)
    assert not np.array_equal(F.p, F.q), "expected row exchanges"
    b = np.random.default_rng(n).random(n)
    x = np.empty(n)
    smlu.ldiv_(x, F, b)
    ctol = max(DENSE_TOL, 8 * np.finfo(float).eps * np.linalg.cond(D))
    assert isapprox(x, np.linalg.solve(D, b), ctol, ctol)
    factor_parity(A, F, rtol=1e-10)
    # refactor with new values (same pattern): pivots chosen afresh
    D2 = _tile_pivoting_matrix(n, 99 + n)
    smlu.lu_(F, sp.csc_matrix(D2))
    smlu.ldiv_(x, F, b)
    ctol = max(DENSE_TOL, 8 * np.finfo(float).eps * np.linalg.cond(D2))
    assert isapprox(x, np.linalg.solve(D2, b), ctol, ctol)
    factor_parity(sp.csc_matrix(D2), F, rtol=1e-10)


def _weak_tile_matrix(n, seed):
    """Dense matrix whose 64x64 diagonal blocks are tiny next to the rows below them: the
    diagonal-tile pivoting of large fronts has to accept pivots that fail the threshold test
    (growth > 1/pivot_tol), which the refactor flags as weak pivots."""
    rng = np.random.default_rng(seed)
    D = rng.random((n, n))
    for b0 in range(0, n, 64):
        b1 = min(n, b0 + 64)
        D[b0:b1, b0:b1] = 1e-2 * rng.random((b1 - b0, b1 - b0)) + 1e-2 * np.eye(b1 - b0)
    return D


def test_weak_pivots_trigger_refinement(gpu, monkeypatch):
    # with the re-pivoting refactor switched off (SMLU_NO_REPIVOT), weak tile
    # pivots are left to the solves: refine=-1 (default) refines only when the factorization
    # flagged weak pivots; the refined solution meets the dense tolerance.
    monkeypatch.setenv("SMLU_NO_REPIVOT", "1")
    n = 700
    D = _weak_tile_matrix(n, 21)
    A = sp.csc_matrix(D)
    b = np.random.default_rng(4).random(n)
    xref = np.linalg.solve(D, b)
    ctol = max(DENSE_TOL, 8 * np.finfo(float).eps * np.linalg.cond(D))
    F0 = smlu.ParallelSparseLU(A, refine=0)
    assert F0.stat("weak") > 0, "expected weak pivots in the diagonal-tile path"
    x0 = np.empty(n)
    smlu.ldiv_(x0, F0, b)
    assert F0.stat("refine_steps") == 0
    F = smlu.ParallelSparseLU(A)
    x = np.empty(n)
    smlu.ldiv_(x, F, b)
    assert F.stat("refine_steps") >= 1
    e0 = np.linalg.norm(x0 - xref) / np.linalg.norm(xref)
    e1 = np.linalg.norm(x - xref) / np.linalg.norm(xref)
    assert e1 <= e0
    assert isapprox(x, xref, ctol, ctol), (e0, e1)
    # well-conditioned factorization: no refinement by default, refine=k forces it
    P = mats.poisson3d(12)
    G = smlu.ParallelSparseLU(P)
    xb = np.empty(P.shape[0])
    smlu.ldiv_(xb, G, np.ones(P.shape[0]))
    assert G.stat("weak") == 0 and G.stat("refine_steps") == 0
    G2 = smlu.ParallelSparseLU(P, refine=2)
    smlu.ldiv_(xb, G2, np.ones(P.shape[0]))
    assert G2.stat("refine_residual") >= 0
    assert isapprox(xb, spla.spsolve(P, np.ones(P.shape[0])), TOL, TOL)


@pytest.mark.parametrize("nel", [50, 200])
def test_nondominant_refinement_stops_on_backward_error(gpu, nel):
    # The reference's sparse FE matrix (test/runtests.jl:12-21) is not diagonally dominant, so the
    # default options (diag_pivot_tol 0.001 < pivot_tol 0.1) arm the automatic refinement.  It must
    # stop on LAPACK dgerfs' rule with a rounding floor: no correction solve once the componentwise
    # backward error max|r|/(|A||x|+|b|) is within 4 unit roundoffs (2^-51), at most one for a
    # well-conditioned matrix.
    rng = np.random.default_rng(100 + nel)
    A = sp.csc_matrix(O.test_matrix(rng, nel, 5))
    n = A.shape[0]
    F = smlu.ParallelSparseLU(A)
    assert F.stat("dominant") == 0
    b = rng.random(n)
    x = np.empty(n)
    smlu.ldiv_(x, F, b)
    steps, berr = F.stat("refine_steps"), F.stat("refine_berr")
    assert 0 <= berr <= 2.0 ** -51, (steps, berr)
    assert steps <= 1, (steps, berr)
    if steps == 1:   # a correction was solved only because the first solve's berr exceeded eps
        F0 = smlu.ParallelSparseLU(A, refine=0)
        x0 = np.empty(n)
        smlu.ldiv_(x0, F0, b)
        r0 = np.abs(A @ x0 - b) / (abs(A) @ np.abs(x0) + np.abs(b))
        assert r0.max() > 2.0 ** -51
    assert isapprox(x, spla.spsolve(A, b), TOL, TOL)


def test_solve_multiple_rhs(gpu):
    # ldiv! with a matrix of right-hand sides: equals column-by-column solves
    A = mats.poisson2d(40)
    n = A.shape[0]
    F = smlu.ParallelSparseLU(A)
    B = np.random.default_rng(8).random((n, 5))
    X = np.empty((n, 5))
    smlu.ldiv_(X, F, B)
    for j in range(5):
        xj = np.empty(n)
        smlu.ldiv_(xj, F, B[:, j])
        assert np.array_equal(xj, X[:, j])
        assert isapprox(xj, spla.spsolve(A, B[:, j]), TOL, TOL)
    with pytest.raises(smlu.DimensionMismatch):
        smlu.ldiv_(np.empty((n, 4)), F, B)


@pytest.mark.parametrize("k,nrhs", [(20, 3), (24, 20)])
def test_solve_multiple_rhs_batched(gpu, k, nrhs):
    # batched multi-RHS kernels (16 columns per launch) on 3D Poisson with large fronts (the
    # 64-column block steps): every column bitwise equal to its single-vector solve; host and
    # device entry points agree; nrhs=20 spans two batches.
    import torch
    A = mats.poisson3d(k)
    n = A.shape[0]
    F = smlu.ParallelSparseLU(A)
    B = np.random.default_rng(9).random((n, nrhs))
    X = np.empty((n, nrhs))
    smlu.ldiv_(X, F, B)
    dB = torch.from_numpy(np.ascontiguousarray(B.T)).cuda()
    dX = torch.empty_like(dB)
    F.solve_multi_device(dX, dB)
    assert np.array_equal(dX.cpu().numpy().T, X)
    for j in range(nrhs):
        xj = np.empty(n)
        smlu.ldiv_(xj, F, B[:, j])
        assert np.array_equal(xj, X[:, j]), j
    assert isapprox(X[:, -1], spla.spsolve(A, B[:, -1]), TOL, TOL)


def test_int32_indices(gpu):
    # SparseMatrixCSC{Float64,Int32} through smlu_create_i32: same factors as the Int64 path
    A = mats.poisson3d(10)
    F64 = smlu.ParallelSparseLU(A)
    F32 = smlu.ParallelSparseLU(A, int32_indices=True)
    assert np.array_equal(F64.p, F32.p) and np.array_equal(F64.q, F32.q)
    assert abs(F64.L - F32.L).max() == 0 and abs(F64.U - F32.U).max() == 0


@pytest.mark.parametrize("nel,cs", [(1, None), (7, None), (57, None), (57, 3), (200, 16)])
def test_chunked_layout_ldiv(gpu, nel, cs):
    # the reference's dense-chunk layout on the GPU.  Same factors as ldiv_, so
    # the solutions agree to rounding; against the oracle's verbatim CPU restatement of the
    # chunked lsolve!/rsolve! on the exported factors at the reference's tolerance.
    rng = np.random.default_rng(100 + nel)
    A = O.test_matrix(rng, nel, 5)
    n = A.shape[0]
    F = smlu.ParallelSparseLU(A)
    smlu.chunked_setup(F, cs)
    b = rng.random(n)
    x = np.empty(n)
    smlu.chunked_ldiv_(x, F, b)
    xr = np.empty(n)
    smlu.ldiv_(xr, F, b)
    assert isapprox(x, xr, TOL, TOL)
    CS = O.ChunkedSolve(F.L, F.U, cs)
    w = (F.Rs * b)[F.p]
    CS.lsolve(w)
    CS.rsolve(w)
    xo = np.empty(n)
    xo[F.q] = w
    assert isapprox(x, xo, TOL, TOL)
    assert isapprox(x, spla.spsolve(A, b), TOL, TOL)
    # after lu! the chunks are refilled (src/SharedMemSparseLU.jl:265-276)
    A2 = O.test_matrix(np.random.default_rng(7 + nel), nel, 5)
    smlu.lu_(F, A2)
    smlu.chunked_ldiv_(x, F, b)
    assert isapprox(x, spla.spsolve(A2, b), TOL, TOL)


def test_chunked_layout_dense_and_refusal(gpu):
    rng = np.random.default_rng(9)
    D = rng.random((64, 64))
    A = sp.csc_matrix(D)
    F = smlu.ParallelSparseLU(A)
    smlu.chunked_setup(F)
    b = rng.random(64)
    x = b.copy()
    smlu.chunked_ldiv_(x, F, x)   # x === b allowed
    assert isapprox(x, np.linalg.solve(D, b), DENSE_TOL, DENSE_TOL)
    with pytest.raises(smlu.DimensionMismatch):
        smlu.chunked_ldiv_(np.empty(63), F, b)


def test_dominance_selects_tile_pivoting(gpu):
    # diagonally dominant input: mid-size fronts take the diagonal-tile path (no row exchanges
    # are needed); a random dense matrix keeps full-candidate pivoting.  Both solve correctly.
    A = mats.poisson3d(12)
    F = smlu.ParallelSparseLU(A)
    assert F.stat("dominant") == 1.0
    b = np.random.default_rng(3).random(A.shape[0])
    x = np.empty_like(b)
    smlu.ldiv_(x, F, b)
    assert isapprox(x, spla.spsolve(A, b), TOL, TOL)
    D = np.random.default_rng(4).random((200, 200))
    G = smlu.ParallelSparseLU(sp.csc_matrix(D))
    assert G.stat("dominant") == 0.0
    y = np.empty(200)
    smlu.ldiv_(y, G, b[:200])
    assert isapprox(y, np.linalg.solve(D, b[:200]), DENSE_TOL, DENSE_TOL)
