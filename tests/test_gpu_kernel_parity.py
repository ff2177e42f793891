"""Every kernel variant of the numeric refactor against the oracle, and the error paths.

* GEMM tile variants.  A launch normally takes the fp64 MFMA 128x128 tile (`k_gemm128_mfma3`,
  the v3 tile) only when it has >= 512 output tiles, which the oracle-sized cases never reach.
  The schedule knobs force each variant on oracle-sized fronts, so the dominant kernel of the
  128^3 refactor (`k_gemm128_mfma3<false, *>`) and its TRSM form (`<true, *>`, growth epilogue)
  are compared with the oracle entry by entry:
    mfma128  SMLU_T128MIN=1, SMLU_SMALLK=0    every GEMM launch on k_gemm128_mfma3, the GEMM-form
                                              TRSM included (by default it runs on k_gemm_k64)
    valu64   SMLU_T128MIN=2^60, SMLU_SMALLK=0 every GEMM launch on the VALU 64x64 tile k_gemm
    default  as shipped (k_gemm_k64 for k <= 64 launches, the MFMA 64x64 tile k_gemm64_mfma for
             k > 64 launches below the 128-tile threshold, fused panels with tile inverses, k_urows)
  (round 5 removed the rocBLAS comparison variant together with the library's vendor GEMM path;
  round 6 removed the comparison-only VALU 128 and MFMA v2 tiles from the library)
* Error paths of the reference surface: SingularException from lu(A) (src/SharedMemSparseLU.jl:74)
  and lu!(F, A) (:247), lu! with a changed pattern (the reallocate branch :252-273), the
  re-pivoting refactor (a zero or weak diagonal-tile pivot re-factors with full-candidate
  pivoting) and the per-refactor dominance check.
"""
import numpy as np
import pytest
import scipy.sparse as sp
import scipy.sparse.linalg as spla

import smlu
from smlu import matrices as mats

from _parity import DENSE_TOL, TOL, factor_parity, isapprox, tile_pivoting_matrix

pytestmark = pytest.mark.gpu

VARIANTS = {
    "default": ({}, {}),
    "mfma128": ({"SMLU_T128MIN": "1", "SMLU_SMALLK": "0"}, {}),
    "valu64": ({"SMLU_T128MIN": str(1 << 60), "SMLU_SMALLK": "0"}, {}),
}


def make(A, variant, monkeypatch, **kw):
    env, opts = VARIANTS[variant]
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    F = smlu.ParallelSparseLU(A, **opts, **kw)
    for k in env:
        monkeypatch.delenv(k)
    return F


def check_variant_ran(F, variant):
    if variant == "mfma128":
        assert F.stat("launches_mfma128") > 0 and F.stat("launches_valu64") == 0
        assert F.stat("launches_k64") == 0
    elif variant == "valu64":
        assert F.stat("launches_valu64") > 0
        assert F.stat("launches_mfma128") == 0 and F.stat("launches_k64") == 0
    assert F.stat("vendor_calls") == 0


@pytest.mark.parametrize("variant", list(VARIANTS))
@pytest.mark.parametrize("N", [16, 24])
def test_poisson3d_nd_gemm_variants(gpu, monkeypatch, N, variant):
    # real ND front sizes (root separator N^2 = 256 / 576 pivots, mode-2 fronts with GEMM-form
    # triangular solves under dominance): every variant must match the oracle
    A = mats.poisson3d(N)
    F = make(A, variant, monkeypatch)
    check_variant_ran(F, variant)
    assert F.stat("fronts_mode2") > 0
    if variant == "mfma128":
        assert F.stat("launches_mfma128_trsm") > 0   # k_gemm128_mfma3<true, *>
    factor_parity(A, F)
    assert np.array_equal(F.p, F.q)
    b = np.random.default_rng(N).random(A.shape[0])
    x = np.empty_like(b)
    smlu.ldiv_(x, F, b)
    assert isapprox(x, spla.spsolve(A, b), TOL, TOL)


@pytest.mark.parametrize("variant", ["default", "mfma128"])
def test_poisson3d_32_nd_oracle(gpu, monkeypatch, variant):
    # the largest oracle case (~2.6 s on one core): root separator of 1024 pivots
    A = mats.poisson3d(32)
    F = make(A, variant, monkeypatch)
    check_variant_ran(F, variant)
    factor_parity(A, F)


def test_mfma_and_valu_tiles_bitwise(gpu, monkeypatch):
    # the MFMA tiles (128 x 128, the one-shot k <= 64 tile and the 64 x 64 tile for k > 64)
    # accumulate each C element in the same k order as the VALU 64 tile, one rounding per
    # multiply-add: the factors are bitwise identical
    A = mats.poisson3d(20)
    Fm = make(A, "mfma128", monkeypatch)
    Fv = make(A, "valu64", monkeypatch)
    Fd = make(A, "default", monkeypatch)   # k <= 64 launches on the one-shot MFMA tile
    assert Fd.stat("launches_k64") > 0
    assert Fd.stat("launches_mfma64") > 0  # k > 64 launches below the 128 threshold: k_gemm64_mfma
    assert np.array_equal(Fv.L.indices, Fm.L.indices)
    assert np.array_equal(Fv.L.data, Fm.L.data)
    assert np.array_equal(Fv.U.data, Fm.U.data)
    assert np.array_equal(Fv.L.data, Fd.L.data)
    assert np.array_equal(Fv.U.data, Fd.U.data)


def _dominant_dense(n, seed):
    rng = np.random.default_rng(seed)
    D = rng.random((n, n))
    D += np.diag(D.sum(axis=1) + 1)
    return D


def _tile_pivoting_matrix(n, seed):
    return tile_pivoting_matrix(n, seed)


@pytest.mark.parametrize("variant", ["mfma128", "valu64"])
def test_dense_fronts_gemm_variants(gpu, monkeypatch, variant):
    # one 700-pivot front (mode 2): the GEMM-form TRSM with the growth epilogue on each tile
    # variant, without and with row interchanges inside the diagonal tiles
    for D, rt in ((_dominant_dense(700, 5), 1e-11), (_tile_pivoting_matrix(1100, 1111), 1e-10)):
        A = sp.csc_matrix(D)
        F = make(A, variant, monkeypatch)
        check_variant_ran(F, variant)
        factor_parity(A, F, rtol=rt)
        b = np.random.default_rng(1).random(D.shape[0])
        x = np.empty_like(b)
        smlu.ldiv_(x, F, b)
        ctol = max(DENSE_TOL, 8 * np.finfo(float).eps * np.linalg.cond(D))
        assert isapprox(x, np.linalg.solve(D, b), ctol, ctol)


# ---- error paths -------------------------------------------------------------------------
def test_singular_structural_raises(gpu):
    # an empty column: lu(A) throws SingularException (src/SharedMemSparseLU.jl:74)
    A = mats.poisson2d(6).tolil()
    A[:, 7] = 0.0
    A = sp.csc_matrix(A)
    A.eliminate_zeros()
    with pytest.raises(smlu.SingularException) as ei:
        smlu.ParallelSparseLU(A)
    assert ei.value.info >= 0


@pytest.mark.parametrize("n", [6, 100, 700])
def test_singular_numerical_raises(gpu, n):
    # a zero row (it stays exactly zero through the elimination): small front (LDS kernel),
    # blocked mode 1 and blocked mode 2 (the re-pivoting refactor runs and still finds the
    # zero pivot)
    D = np.random.default_rng(n).random((n, n))
    D[n - 2, :] = 0.0
    with pytest.raises(smlu.SingularException):
        smlu.ParallelSparseLU(sp.csc_matrix(D))


def test_singular_in_refactor_raises(gpu):
    # lu!(F, A) with singular values of the same pattern throws too (:247)
    A = mats.poisson2d(8)
    F = smlu.ParallelSparseLU(A)
    A2 = A.tocsr()
    A2.data[A2.indptr[20]:A2.indptr[21]] = 0.0   # row 20 zero (stored zeros: same pattern)
    A2 = A2.tocsc()
    assert A2.nnz == A.nnz
    with pytest.raises(smlu.SingularException):
        smlu.lu_(F, A2)


@pytest.mark.parametrize("where", [0, 100])
def test_zero_diagonal_block(gpu, where):
    # nonsingular matrix with a zero 64x64 diagonal block: the fronts pivot only among their
    # fully-summed rows (UMFPACK's column pivoting has no such limit), so the analysis first
    # permutes rows for a zero-free diagonal (maximum transversal); then the factors match the
    # oracle and the solve meets the dense tolerance
    n = 700
    rng = np.random.default_rng(17)
    D = rng.random((n, n))
    D[where:where + 64, where:where + 64] = 0.0
    A = sp.csc_matrix(D)
    F = smlu.ParallelSparseLU(A)
    assert F.stat("matched") == 1
    assert not np.array_equal(F.p, F.q)
    b = rng.random(n)
    x = np.empty(n)
    smlu.ldiv_(x, F, b)
    ctol = max(DENSE_TOL, 8 * np.finfo(float).eps * np.linalg.cond(D))
    assert isapprox(x, np.linalg.solve(D, b), ctol, ctol)
    factor_parity(A, F, rtol=1e-9)


def test_kkt_zero_block(gpu):
    # saddle-point matrix [[H, B'], [B, 0]] with a 300x300 zero block, one 1000-pivot front
    rng = np.random.default_rng(23)
    m, k = 700, 300
    H = rng.random((m, m)); H = H + H.T + m * np.eye(m)
    B = rng.random((k, m))
    D = np.block([[H, B.T], [B, np.zeros((k, k))]])
    A = sp.csc_matrix(D)
    F = smlu.ParallelSparseLU(A)
    assert F.stat("matched") == 1
    b = rng.random(m + k)
    x = np.empty(m + k)
    smlu.ldiv_(x, F, b)
    ctol = max(DENSE_TOL, 8 * np.finfo(float).eps * np.linalg.cond(D))
    assert isapprox(x, np.linalg.solve(D, b), ctol, ctol)


def test_full_candidate_tall_panels(gpu, monkeypatch):
    # the panels of the re-pivoting refactor with more than 512 candidate rows (k_panel_tall),
    # forced on a random dense front: oracle parity with the GPU's own pivot sequence
    D = np.random.default_rng(17).random((700, 700))
    A = sp.csc_matrix(D)
    monkeypatch.setenv("SMLU_FULLPIV_NS", "100000")
    F = smlu.ParallelSparseLU(A, diag_pivot_tol=0.1)   # exchanges on most columns
    monkeypatch.delenv("SMLU_FULLPIV_NS")
    assert F.stat("launches_panel_tall") > 0 and F.stat("fronts_mode2") == 0
    factor_parity(A, F, rtol=1e-10, full_piv_ns=100000)
    b = np.random.default_rng(1).random(700)
    x = np.empty(700)
    smlu.ldiv_(x, F, b)
    ctol = max(DENSE_TOL, 8 * np.finfo(float).eps * np.linalg.cond(D))
    assert isapprox(x, np.linalg.solve(D, b), ctol, ctol)


def _weak_tile_matrix(n, seed):
    rng = np.random.default_rng(seed)
    D = rng.random((n, n))
    for b0 in range(0, n, 64):
        b1 = min(n, b0 + 64)
        D[b0:b1, b0:b1] = 1e-2 * rng.random((b1 - b0, b1 - b0)) + 1e-2 * np.eye(b1 - b0)
    return D


@pytest.mark.parametrize("variant", ["default", "mfma128"])
def test_weak_tile_pivots_repivot(gpu, monkeypatch, variant):
    # weak diagonal-tile pivots (growth flagged by the GEMM-form TRSM epilogue) trigger the
    # re-pivoting refactor: full-candidate pivots, no weak pivot left, no refinement needed.  The
    # fallback machinery at the tile pivoting's design tolerance (diag_pivot_tol 0.1): under
    # UMFPACK's 0.001 this adversarial matrix keeps its 0.01 diagonals and grows like UMFPACK does
    D = _weak_tile_matrix(700, 21)
    A = sp.csc_matrix(D)
    F = make(A, variant, monkeypatch, diag_pivot_tol=0.1)
    assert F.stat("repivots") == 1
    assert F.stat("weak") == 0
    b = np.random.default_rng(4).random(700)
    x = np.empty(700)
    smlu.ldiv_(x, F, b)
    assert F.stat("refine_steps") == 0
    ctol = max(DENSE_TOL, 8 * np.finfo(float).eps * np.linalg.cond(D))
    assert isapprox(x, np.linalg.solve(D, b), ctol, ctol)
    factor_parity(A, F, rtol=1e-10)


def test_dominant_then_nondominant_refactor(gpu):
    # created with dominant values (mid-size fronts take diagonal-tile pivoting), then lu! with
    # values of the same pattern that are far from dominant: the refactor re-checks dominance
    # and the mid-size fronts pivot over all fully-summed rows again
    A = mats.poisson3d(12)
    F = smlu.ParallelSparseLU(A)
    assert F.stat("dominant") == 1.0
    m2 = F.stat("fronts_mode2")
    assert m2 > 0
    A2 = A.copy()
    A2.data = np.random.default_rng(9).standard_normal(A.nnz)
    smlu.lu_(F, A2)
    assert F.stat("dominant") == 0.0
    assert F.stat("fronts_mode2") < m2
    b = np.random.default_rng(2).random(A.shape[0])
    x = np.empty_like(b)
    smlu.ldiv_(x, F, b)
    xr = spla.spsolve(A2, b)
    ctol = max(TOL, 8 * np.finfo(float).eps * np.linalg.cond(A2.toarray()))
    assert isapprox(x, xr, ctol, ctol)
    factor_parity(A2, F, rtol=1e-9)
    # and back to dominant values: the fast schedule returns
    smlu.lu_(F, mats.perturb_diag(A, 3))
    assert F.stat("dominant") == 1.0 and F.stat("fronts_mode2") == m2


def test_lu_pattern_change(gpu):
    # lu!(F, A) with a different pattern: the reallocate branch (:252-273) re-analyses;
    # the new (unsymmetric) pattern's factors match the oracle exactly in pattern
    A = mats.poisson2d(12)
    F = smlu.ParallelSparseLU(A)
    n = A.shape[0]
    rng = np.random.default_rng(31)
    E = sp.random(n, n, density=0.01, random_state=np.random.RandomState(3), format="csc")
    A2 = sp.csc_matrix(A + E + sp.eye(n) * 4)
    assert A2.nnz != A.nnz
    smlu.lu_(F, A2)
    factor_parity(A2, F, rtol=1e-11)
    b = rng.random(n)
    x = np.empty(n)
    smlu.ldiv_(x, F, b)
    assert isapprox(x, spla.spsolve(A2, b), TOL, TOL)
    # and back to the original pattern
    smlu.lu_(F, A)
    smlu.ldiv_(x, F, b)
    assert isapprox(x, spla.spsolve(A, b), TOL, TOL)


def test_refactor_device_redecides_pivoting_mode(gpu):
    # the device-only lu! (values already in HBM, the bench's usage) re-checks dominance on the
    # GPU (k_dominance) like the host lu! does: after a re-pivoting refactor left the handle in
    # full-candidate mode, dominant values bring the fast diagonal-tile schedule back
    import torch
    n = 700
    Dd = _dominant_dense(n, 41)
    A = sp.csc_matrix(Dd)
    F = smlu.ParallelSparseLU(A, diag_pivot_tol=0.1)   # the weak-tile matrix below: see above
    assert F.stat("dominant") == 1.0 and F.stat("pivmode") == 0
    m2 = F.stat("fronts_mode2")
    assert m2 > 0

    def dev(D):
        return torch.tensor(sp.csc_matrix(D).data, dtype=torch.float64, device="cuda")

    Dw = _weak_tile_matrix(n, 42)
    F.refactor_device(dev(Dw))
    assert F.stat("dominant") == 0.0
    assert F.stat("repivots") == 1 and F.stat("pivmode") == 1 and F.stat("weak") == 0
    # one synchronisation per refactor: the dominance flags came back in the factorization's status
    # record, the values were factored in the old mode first and again in the new one
    assert F.stat("mode_refactors") == 1
    b = np.random.default_rng(5).random(n)
    x = np.empty(n)
    smlu.ldiv_(x, F, b)
    ctol = max(DENSE_TOL, 8 * np.finfo(float).eps * np.linalg.cond(Dw))
    assert isapprox(x, np.linalg.solve(Dw, b), ctol, ctol)
    factor_parity(sp.csc_matrix(Dw), F, rtol=1e-10)
    Dd2 = _dominant_dense(n, 43)
    F.refactor_device(dev(Dd2))
    assert F.stat("dominant") == 1.0 and F.stat("pivmode") == 0
    assert F.stat("fronts_mode2") == m2 and F.stat("repivots") == 1 and F.stat("mode_refactors") == 2
    # same values again: no mode change, no second factorization
    F.refactor_device(dev(Dd2))
    assert F.stat("mode_refactors") == 2
    # lu! with host values (smlu_refactor: upload + the same device path) gives the same factors
    Ld, Ud = F.L.copy(), F.U.copy()
    F.refactor(sp.csc_matrix(Dd2).data)
    assert np.array_equal(F.L.data, Ld.data) and np.array_equal(F.U.data, Ud.data)
    smlu.ldiv_(x, F, b)
    assert isapprox(x, np.linalg.solve(Dd2, b), DENSE_TOL, DENSE_TOL)
    factor_parity(sp.csc_matrix(Dd2), F, rtol=1e-11)
