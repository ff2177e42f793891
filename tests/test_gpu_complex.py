"""ComplexF64 on the GPU (the reference is generic in Tf,
src/SharedMemSparseLU.jl:43, :64, :286).  The library factors the real-equivalent K of a complex
A (include/smlu.h smlu_create_z); checked here against
  * the oracle's LU of K (oracle.real_equivalent) with the GPU's own (p, q): Rs bitwise, L/U
    pattern bit-identical, values to 1e-12 (1e-10 where pivots are chosen among near ties);
  * scipy's complex SuperLU for the complex solutions, at the reference's sparse tolerance
    1e-12 (or 8 eps kappa(A) when larger, written as ctol).
Covers the FE fixture with complex values, shifted 3D Laplacians up to 24^3 (ND root separator
of 576 complex = 1152 real pivots: blocked fronts, MFMA tiles), a purely imaginary diagonal (row
interchanges inside the 2x2 blocks), lu! (same and changed pattern), device-resident values and
vectors, several right-hand sides, lsolve!/rsolve! and the singular path."""
import numpy as np
import pytest
import scipy.sparse as sp
import scipy.sparse.linalg as spla

import oracle as O
import smlu
from smlu import matrices as mats

from _parity import TOL, factor_parity, isapprox
from test_oracle import complex_fe

pytestmark = pytest.mark.gpu


def ctol(A, tol=TOL):
    if A.shape[0] > 3000:
        return tol
    return max(tol, 8 * np.finfo(float).eps * np.linalg.cond(A.toarray()))


def crand(rng, n):
    return rng.random(n) - 0.5 + 1j * (rng.random(n) - 0.5)


def helmholtz3d(N, shift=1.0):
    """Shifted 7-point Laplacian: -Delta + i*shift*I (complex symmetric, non-Hermitian)."""
    A = mats.poisson3d(N).astype(np.complex128)
    A = (A + 1j * shift * sp.identity(A.shape[0], format="csc")).tocsc()
    A.sort_indices()
    return A


def check_solve(F, A, rng, tol=None):
    n = A.shape[0]
    b = crand(rng, n)
    x = np.empty(n, np.complex128)
    smlu.ldiv_(x, F, b)
    xs = spla.spsolve(A.tocsc(), b)
    assert isapprox(x, xs, tol or ctol(A), tol or ctol(A)), np.linalg.norm(x - xs) / np.linalg.norm(xs)
    return x


@pytest.mark.parametrize("nel", [1, 5, 40])
def test_complex_fe(gpu, nel):
    rng = np.random.default_rng(nel)
    A = complex_fe(rng, nel)
    F = smlu.ParallelSparseLU(A)
    assert F.is_complex and F.stat("complex") == 1
    factor_parity(O.real_equivalent(A), F)
    check_solve(F, A, rng)


@pytest.mark.parametrize("N,grid", [(8, True), (16, False), (24, True)])
def test_complex_helmholtz3d(gpu, N, grid):
    A = helmholtz3d(N, shift=0.5)
    F = smlu.ParallelSparseLU(A, grid=(N, N, N) if grid else None)
    K = O.real_equivalent(A)
    factor_parity(K, F, rtol=1e-10)
    # the column order keeps each complex column's two real columns together
    q = F.real_equivalent_factors()["q"]
    assert np.array_equal(q[0::2] // 2, q[1::2] // 2)
    check_solve(F, A, np.random.default_rng(N), tol=1e-11)


def test_complex_imaginary_diagonal(gpu):
    """Purely imaginary diagonal: K's 2x2 diagonal blocks [[0, -y], [y, 0]] force row interchanges
    inside the blocks."""
    rng = np.random.default_rng(5)
    P = mats.poisson2d(20).astype(np.complex128)
    A = P.copy()
    A.data = np.where(A.indices == np.repeat(np.arange(A.shape[0]), np.diff(A.indptr)),
                      1j * P.data, 0.1 * crand(rng, P.nnz))
    A = sp.csc_matrix(A)
    F = smlu.ParallelSparseLU(A)
    factor_parity(O.real_equivalent(A), F, rtol=1e-10)
    fk = F.real_equivalent_factors()
    assert not np.array_equal(fk["p"], fk["q"])   # interchanges happened
    # the pair rule keeps every complex row pair (swapped inside where |Im| > |Re|), so the complex
    # factors exist (round 4; rounds 1-3 split the pairs here and F.L raised)
    pk = fk["p"]
    assert (pk[0::2] > pk[1::2]).any()
    _check_complex_factors(A, F)
    check_solve(F, A, rng)


def test_complex_random_dominant(gpu):
    rng = np.random.default_rng(11)
    R = mats.random_dominant(400, 0.02, seed=3).astype(np.complex128)
    R.data = R.data * np.exp(1j * rng.random(R.nnz) * 2 * np.pi)
    A = sp.csc_matrix(R)
    F = smlu.ParallelSparseLU(A)
    factor_parity(O.real_equivalent(A), F, rtol=1e-10)
    check_solve(F, A, rng)


def test_complex_refactor_same_and_new_pattern(gpu):
    rng = np.random.default_rng(21)
    A = complex_fe(rng, 30)
    F = smlu.ParallelSparseLU(A)
    A2 = A.copy()
    A2.data = A2.data * (1 + 0.3 * crand(rng, A2.nnz))
    smlu.lu_(F, A2)
    factor_parity(O.real_equivalent(A2), F)
    check_solve(F, A2, rng)
    A3 = A2.tolil()                          # changed pattern: re-analysis (:252-273)
    n = A3.shape[0]
    A3[0, n - 1] = 0.01 + 0.02j
    A3[n - 1, 0] = -0.01j
    A3 = sp.csc_matrix(A3)
    A3.sort_indices()
    smlu.lu_(F, A3)
    factor_parity(O.real_equivalent(A3), F)
    check_solve(F, A3, rng)


def test_complex_device_paths(gpu):
    import torch
    rng = np.random.default_rng(31)
    A = helmholtz3d(10, shift=2.0)
    n = A.shape[0]
    F = smlu.ParallelSparseLU(A)
    A2 = A.copy()
    A2.data = A2.data + 0.25 * crand(rng, A2.nnz)
    dv = torch.from_numpy(A2.data.copy()).to("cuda:0")
    F.refactor_device(dv)
    torch.cuda.synchronize()
    factor_parity(O.real_equivalent(A2), F)
    b = crand(rng, n)
    db = torch.from_numpy(b).to("cuda:0")
    dx = torch.empty_like(db)
    F.solve_device(dx, db)
    torch.cuda.synchronize()
    x = dx.cpu().numpy()
    assert isapprox(x, spla.spsolve(A2, b), TOL, TOL)
    # several right-hand sides on the device, (nrhs, n) complex
    B = np.stack([crand(rng, n) for _ in range(5)])
    dB = torch.from_numpy(B).to("cuda:0")
    dX = torch.empty_like(dB)
    F.solve_multi_device(dX, dB)
    torch.cuda.synchronize()
    X = dX.cpu().numpy()
    for r in range(5):
        assert isapprox(X[r], spla.spsolve(A2, B[r]), TOL, TOL)


def test_complex_multi_rhs_host_and_aliasing(gpu):
    rng = np.random.default_rng(41)
    A = complex_fe(rng, 25)
    n = A.shape[0]
    F = smlu.ParallelSparseLU(A)
    B = np.asfortranarray(np.stack([crand(rng, n) for _ in range(7)], axis=1))
    X = np.empty_like(B)
    smlu.ldiv_(X, F, B)
    Xs = spla.spsolve(A, B)
    for r in range(7):
        assert isapprox(X[:, r], Xs[:, r], ctol(A), ctol(A))
    b = crand(rng, n)
    x = b.copy()
    smlu.ldiv_(x, F, x)                      # x === b allowed (:286)
    assert isapprox(x, spla.spsolve(A, b), ctol(A), ctol(A))


def test_complex_lsolve_rsolve(gpu):
    rng = np.random.default_rng(51)
    A = complex_fe(rng, 12)
    n = A.shape[0]
    F = smlu.ParallelSparseLU(A)
    b = crand(rng, n)
    x = b.copy()
    smlu.lsolve_(F, x)
    fk = F.real_equivalent_factors()
    ref = spla.spsolve_triangular(fk["L"].tocsr(), b.view(np.float64), lower=True)
    assert isapprox(x.view(np.float64), ref, TOL, TOL)
    x = b.copy()
    smlu.rsolve_(F, x)
    ref = spla.spsolve_triangular(fk["U"].tocsr(), b.view(np.float64), lower=False)
    assert isapprox(x.view(np.float64), ref, 1e-10, 1e-10)


def test_complex_singular(gpu):
    rng = np.random.default_rng(61)
    A = complex_fe(rng, 6).tolil()
    A[:, 4] = 0                               # a zero column: structurally singular
    A = sp.csc_matrix(A)
    A.eliminate_zeros()
    with pytest.raises(smlu.SingularException):
        smlu.ParallelSparseLU(A)


def test_complex_type_checks(gpu):
    A = mats.poisson2d(5)
    F = smlu.ParallelSparseLU(A)
    with pytest.raises(TypeError):
        smlu.ldiv_(np.empty(25, np.complex128), F, np.ones(25, np.complex128))
    with pytest.raises(TypeError):
        smlu.lu_(F, A.astype(np.complex128) * 1j)


def _check_complex_factors(A, F):
    """F.L, F.U, F.p, F.q, F.Rs of a complex handle are complex n x n (the reference's
    SparseMatrixCSC{ComplexF64}, src/SharedMemSparseLU.jl:47-52): UMFPACK's conventions (L unit
    diagonal stored first, U diagonal last, rows sorted) and L*U == (Rs.*A)[p, q]; they fold the
    real-equivalent factors exactly (Rs of complex row i = Rs of K's row 2i; row 2i+1 agrees to rounding)."""
    L, U, p, q, Rs = F.L, F.U, F.p, F.q, F.Rs
    n = A.shape[0]
    assert L.dtype == np.complex128 and U.dtype == np.complex128 and L.shape == (n, n)
    fk = F.real_equivalent_factors()
    assert np.array_equal(p, fk["p"][0::2] // 2) and np.array_equal(q, fk["q"][0::2] // 2)
    assert np.array_equal(Rs, fk["Rs"][0::2])
    # K's rows 2i and 2i+1 sum the same magnitudes |Re a_ij|, |Im a_ij| in swapped order per j:
    # equal to the last bits only
    assert np.allclose(fk["Rs"][0::2], fk["Rs"][1::2], rtol=1e-14, atol=0)
    for j in range(n):
        li = L.indices[L.indptr[j]:L.indptr[j + 1]]
        ui = U.indices[U.indptr[j]:U.indptr[j + 1]]
        assert li[0] == j and L.data[L.indptr[j]] == 1.0 and np.all(np.diff(li) > 0)
        assert ui[-1] == j and np.all(np.diff(ui) > 0)
    B = (sp.diags(Rs) @ A).tocsr()[p][:, q]
    E = L @ U - B
    assert abs(E).max() <= 1e-12 * max(abs(B).max(), 1.0)


@pytest.mark.parametrize("case", ["helmholtz", "dominant", "fe"])
def test_complex_factor_export(gpu, case):
    rng = np.random.default_rng(71)
    if case == "helmholtz":
        A = helmholtz3d(12, shift=0.5)
    elif case == "dominant":
        R = mats.random_dominant(300, 0.02, seed=9).astype(np.complex128)
        # random phases off the diagonal only: a diagonal entry near the imaginary axis makes the
        # real-equivalent 2x2 block [[a, -b], [b, a]] swap its rows (|b| > 10|a|), which splits
        # the pair (covered by the "fe" case and test_imaginary_diagonal*)
        R = sp.coo_matrix(R)
        off = R.row != R.col
        R.data[off] = R.data[off] * np.exp(1j * rng.random(off.sum()) * 2 * np.pi)
        A = sp.csc_matrix(R)
    else:
        A = complex_fe(rng, 20)
    F = smlu.ParallelSparseLU(A)
    fk = F.real_equivalent_factors()
    pk = fk["p"]
    # pair-preserving pivots (round 4): every complex row pair stays adjacent, in either order
    paired = np.all(np.minimum(pk[0::2], pk[1::2]) % 2 == 0) and np.all(np.abs(pk[0::2] - pk[1::2]) == 1)
    assert paired
    assert F.stat("cpair") == 1
    _check_complex_factors(A, F)
