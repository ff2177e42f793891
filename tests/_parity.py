"""Shared parity helpers of the GPU tests: the oracle comparison of exported factors and the
reference's isapprox (test/runtests.jl:25-26 tolerances)."""
import numpy as np
import scipy.sparse as sp

import oracle as O

TOL = 1.0e-12
DENSE_TOL = 1.0e-10


def isapprox(x, y, rtol, atol):
    """Julia's isapprox for vectors: norm(x-y) <= max(atol, rtol*max(norm(x), norm(y)))."""
    return np.linalg.norm(x - y) <= max(atol, rtol * max(np.linalg.norm(x), np.linalg.norm(y)))


def assert_same_pattern(G, R):
    """CSC colptr and rowval identical (stored entries, explicit zeros included)."""
    assert G.shape == R.shape
    assert np.array_equal(G.indptr, R.indptr), "colptr differs from the oracle's"
    assert np.array_equal(G.indices, R.indices), "rowval differs from the oracle's"


def _real(F):
    """The factors the GPU holds (a complex handle: those of its real-equivalent K)."""
    return F.real_equivalent_factors() if getattr(F, "is_complex", False) else \
        dict(L=F.L, U=F.U, p=F.p, q=F.q, Rs=F.Rs)


def pivot_parity(A, F, prev_pivmode=0, full_piv_ns=None, given=False):
    """The GPU's pivot DECISIONS against an independent restatement of its rule: the multifrontal
    oracle (oracle/mf.c) chooses its own row order on the handle's assembly tree (threshold
    partial pivoting with diagonal preference inside each front's candidate rows, the candidate
    modes and the re-pivoting refactor restated in oracle.gpu_pivot_choice).  p must be
    bit-identical; so must the per-front candidate modes and the final pivoting mode."""
    fr = F.fronts()
    fx = _real(F)
    p_or, pm, modes, _ = O.gpu_pivot_choice(A, fx["q"], fr, pivmode=prev_pivmode, full_piv_ns=full_piv_ns,
                                            given=given, pivot_tol=F.stat("pivot_tol"),
                                            diag_tol=F.stat("diag_pivot_tol") if not given else 0.1,
                                            pairs=F.stat("cpair") == 1)
    assert np.array_equal(modes, fr["mode"]), "per-front pivot candidate modes differ from the restated rule"
    assert int(F.stat("pivmode")) == pm, (F.stat("pivmode"), pm)
    bad = np.flatnonzero(np.asarray(fx["p"]) != p_or)
    assert bad.size == 0, f"pivot order differs from the oracle's at {bad.size} positions, first {bad[:8]}"
    return p_or


def factor_parity(A, F, rtol=1e-12, prev_pivmode=0, full_piv_ns=None):
    """Pivot order chosen independently by the multifrontal oracle (pivot_parity), then the
    exported factors vs the oracle's fixed-pivot LU of (Rs.*A)[p, q]."""
    pivot_parity(A, F, prev_pivmode=prev_pivmode, full_piv_ns=full_piv_ns)
    fx = _real(F)
    p, q, Rs = fx["p"], fx["q"], fx["Rs"]
    Ro = O.rowscale(A)
    assert np.array_equal(Rs, Ro), "row scaling must be bitwise identical"
    ref = O.OracleLU(A, p, q, Ro)
    assert ref.status == 0
    L, U = fx["L"], fx["U"]
    B = (sp.diags(Rs) @ A).tocsr()[p][:, q]
    # the tolerance scales with the growth factor rho = max|U| / max|(Rs.*A)[p,q]|: two correctly
    # rounded LUs with the same pivots differ by about n eps rho max|A| (Wilkinson), and a
    # diagonal kept under UMFPACK's symmetric tolerance 0.001 lets non-dominant fronts grow
    rho = max(1.0, abs(ref.U).max() / max(abs(B).max(), 1e-300))
    for G, R in ((L, ref.L), (U, ref.U)):
        # pattern: bit-identical colptr/rowval to the oracle's structural fill of (Rs.*A)[p,q]
        assert_same_pattern(G, R)
        D = (G - R)
        scale = max(abs(R).max(), 1.0)
        assert abs(D).max() <= rtol * rho * scale, f"factor mismatch {abs(D).max()} (scale {scale}, growth {rho})"
    # UMFPACK contract L*U == (Rs.*A)[p,q]
    E = L @ U - B
    assert abs(E).max() <= 1e-10 * max(abs(B).max(), 1.0)
    return ref


def tile_pivoting_matrix(n, seed):
    """Dense matrix whose 64x64 diagonal blocks dominate their rows but whose diagonal entries are
    tiny (below 0.001 x the tile's column maxima, so rows are exchanged under UMFPACK's symmetric
    diagonal tolerance as well): the diagonal-tile panel (mode 2, ns > 512) must exchange rows
    inside every tile."""
    rng = np.random.default_rng(seed)
    D = rng.random((n, n))
    for b0 in range(0, n, 64):
        b1 = min(n, b0 + 64)
        blk = rng.random((b1 - b0, b1 - b0)) * n
        np.fill_diagonal(blk, 1e-3)
        D[b0:b1, b0:b1] += blk
    np.fill_diagonal(D, 1e-3 * rng.random(n))
    return D


def front_parity(A, F, rtol=1e-12, threads=16, prev_pivmode=0):
    """Factor parity at sizes the one-core fixed-pivot oracle cannot reach: the multifrontal oracle
    (oracle/mf.c, OpenMP) chooses its own pivots on the handle's assembly tree (the candidate modes
    and the re-pivoting decision restated as in pivot_parity: modes, pivmode and p bit-identical,
    Rs bitwise), then EVERY front's stored factor values -- its L panel (M x ns: unit-lower
    multipliers and U11) and U12 (ns x nu) -- are compared entry by entry with the GPU's factor
    store (smlu_dev_front_offsets / smlu_dev_copy).  Tolerance per front: rtol * growth * max(1,
    max |front|).  Returns (fronts compared, entries compared, worst scaled difference)."""
    A = sp.csc_matrix(A)
    A.sort_indices()
    fr = F.fronts()
    p, q, Rs = F.perm_scale()
    assert np.array_equal(Rs, O.rowscale(A)), "row scaling must be bitwise identical"
    p_or, pm, modes, _, mf = O.gpu_pivot_choice(A, q, fr, pivmode=prev_pivmode, pivot_tol=F.stat("pivot_tol"),
                                                diag_tol=F.stat("diag_pivot_tol"), threads=threads, keep=True)
    try:
        assert np.array_equal(modes, fr["mode"]), "per-front pivot candidate modes differ from the restated rule"
        assert int(F.stat("pivmode")) == pm, (F.stat("pivmode"), pm)
        bad = np.flatnonzero(p != p_or)
        assert bad.size == 0, f"pivot order differs from the oracle's at {bad.size} positions, first {bad[:8]}"
        store, off = F.front_store()
        nsz = np.diff(fr["first"])
        nuz = np.diff(fr["rowptr"])
        amax = max(abs(A.data).max() * abs(Rs).max(), 1e-300)
        worst, entries = 0.0, 0
        for s in range(nsz.size):
            ns_, nu_ = int(nsz[s]), int(nuz[s])
            M = ns_ + nu_
            G = np.concatenate([store[off[s, 0]:off[s, 0] + M * ns_], store[off[s, 1]:off[s, 1] + ns_ * nu_]])
            R = mf.front_values(s)
            assert G.size == R.size
            rmax = abs(R).max() if R.size else 0.0
            rho = max(1.0, rmax / amax)
            d = abs(G - R).max() / (rho * max(rmax, 1.0)) if R.size else 0.0
            assert d <= rtol, f"front {s} (ns {ns_}, nu {nu_}, mode {fr['mode'][s]}): scaled difference {d:.3g}"
            worst = max(worst, d)
            entries += R.size
        return nsz.size, entries, worst
    finally:
        mf.close()
