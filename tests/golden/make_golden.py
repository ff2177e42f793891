"""Generate the committed golden fixtures (tests/golden/*.npz).

Each fixture holds INPUTS (A in CSC, the pivot order p, q, a right-hand side b) and EXPECTED
OUTPUTS (Rs, L, U in CSC, x = A \\ b) of the fixed-pivot oracle (oracle/oracle.c).  Before a
fixture is written, the oracle's outputs are cross-checked against third-party references
available in this image: LAPACK via scipy.linalg.lu for dense cases (same pivots => same L,U),
SuperLU via scipy.sparse.linalg.spsolve for the solution vectors, and the UMFPACK relation
L*U == (Rs.*A)[p,q] (src/SharedMemSparseLU.jl:305-316).  The reference itself (Julia +
UMFPACK) cannot run here, so these vectors pin the oracle, not UMFPACK's pivot order.

The C1 fixture (tests/golden/c1/) holds digests of L and U instead of the full factors (size).

Run:  python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np
import scipy.linalg as sla
import scipy.sparse as sp
import scipy.sparse.linalg as spla

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "sharedmemsparselu.jl_amd"))

import oracle as O  # noqa: E402
from smlu import matrices as mats  # noqa: E402
from smlu.plan import Plan  # noqa: E402


def save(name, A, p, q, b, check_dense_lu=False):
    A = sp.csc_matrix(A)
    A.sort_indices()
    F = O.OracleLU(A, p, q)
    assert F.status == 0
    x = np.empty(A.shape[0])
    F.ldiv(x, b)
    # cross-checks
    B = (sp.diags(F.Rs) @ A).tocsr()[p][:, q]
    assert abs(F.L @ F.U - B).max() <= 1e-12 * max(1.0, abs(B).max())
    xs = spla.spsolve(A, b)
    assert np.linalg.norm(x - xs) <= 1e-9 * max(1.0, np.linalg.norm(xs)), name
    if check_dense_lu:
        Pm, Ls, Us = sla.lu(B.toarray())
        assert np.allclose(Pm, np.eye(A.shape[0]))  # p already holds LAPACK's pivots
        assert np.allclose(F.L.toarray(), Ls, rtol=1e-13, atol=1e-14)
        assert np.allclose(F.U.toarray(), Us, rtol=1e-13, atol=1e-14)
    np.savez_compressed(os.path.join(HERE, name + ".npz"),
                        A_indptr=A.indptr.astype(np.int64), A_indices=A.indices.astype(np.int64),
                        A_data=A.data, n=A.shape[0], p=np.asarray(p, np.int64), q=np.asarray(q, np.int64),
                        b=b, Rs=F.Rs, x=x,
                        L_indptr=F.L.indptr, L_indices=F.L.indices, L_data=F.L.data,
                        U_indptr=F.U.indptr, U_indices=F.U.indices, U_data=F.U.data)
    print("wrote", name, A.shape[0], F.L.nnz, F.U.nnz)


def lapack_rows(A):
    """Row order chosen by LAPACK partial pivoting on Rs.*A (q = identity)."""
    Rs = O.rowscale(A)
    D = (sp.diags(Rs) @ A).toarray()
    P, _, _ = sla.lu(D)
    return np.argmax(P, axis=0)   # row of A placed at position k


def pattern_hash(M):
    """sha256 of a CSC pattern (colptr and rowval as little-endian int64)."""
    import hashlib
    h = hashlib.sha256()
    h.update(np.ascontiguousarray(M.indptr, dtype="<i8").tobytes())
    h.update(np.ascontiguousarray(M.indices, dtype="<i8").tobytes())
    return h.hexdigest()


def factor_digest(M, pick):
    """Compact expected values of a large factor: per-column sums, sums of squares, and the values
    at `pick` (entry positions in CSC storage order)."""
    cs = np.add.reduceat(M.data, M.indptr[:-1]) if M.nnz else np.zeros(M.shape[1])
    cs[np.diff(M.indptr) == 0] = 0.0
    sq = np.add.reduceat(M.data * M.data, M.indptr[:-1]) if M.nnz else np.zeros(M.shape[1])
    sq[np.diff(M.indptr) == 0] = 0.0
    return cs, sq, M.data[pick]


def save_c1(name, A, q, b):
    """the C1 configuration (n=1000, 1 % Bernoulli pattern, U(0,1) values,
    default_rng(47), dominant diagonal) with the plan's default column order q and p = q (a
    dominant matrix keeps every diagonal pivot).  Its 5.5e5 factor entries would make a 5 MB
    fixture, so L and U are pinned by their pattern hashes, nnz, per-column sums and sums of
    squares, and 4096 sampled entries; Rs, x in full."""
    A = sp.csc_matrix(A)
    A.sort_indices()
    F = O.OracleLU(A, q, q)
    assert F.status == 0
    x = np.empty(A.shape[0])
    F.ldiv(x, b)
    B = (sp.diags(F.Rs) @ A).tocsr()[q][:, q]
    assert abs(F.L @ F.U - B).max() <= 1e-12 * max(1.0, abs(B).max())
    xs = spla.spsolve(A, b)
    assert np.linalg.norm(x - xs) <= 1e-10 * max(1.0, np.linalg.norm(xs)), name
    lu = spla.splu(A, permc_spec="NATURAL", diag_pivot_thresh=0.0)   # SuperLU on the same order
    assert np.linalg.norm(lu.solve(b) - x) <= 1e-10 * np.linalg.norm(x)
    prng = np.random.default_rng(1000)
    out = dict(A_indptr=A.indptr.astype(np.int64), A_indices=A.indices.astype(np.int64), A_data=A.data,
               n=A.shape[0], p=np.asarray(q, np.int64), q=np.asarray(q, np.int64), b=b, Rs=F.Rs, x=x)
    for tag, M in (("L", F.L), ("U", F.U)):
        pick = np.sort(prng.choice(M.nnz, 4096, replace=False))
        cs, sq, vals = factor_digest(M, pick)
        out.update({f"{tag}_hash": pattern_hash(M), f"{tag}_nnz": M.nnz, f"{tag}_colsum": cs,
                    f"{tag}_colsq": sq, f"{tag}_pick": pick, f"{tag}_pickval": vals})
    os.makedirs(os.path.join(HERE, "c1"), exist_ok=True)
    np.savez_compressed(os.path.join(HERE, "c1", name + ".npz"), **out)
    print("wrote", name, A.shape[0], F.L.nnz, F.U.nnz)


def main():
    rng = np.random.default_rng(20241020)
    for n in (1, 2, 3, 5, 8, 13):
        A = sp.csc_matrix(rng.random((n, n)))
        p = lapack_rows(A)
        save(f"dense_{n}", A, p, np.arange(n), rng.random(n), check_dense_lu=True)
    for nel in (1, 2, 5, 8):
        A = O.test_matrix(rng, nel, 5)
        n = A.shape[0]
        p = lapack_rows(A)   # FE matrices are not diagonally dominant: use LAPACK's rows
        save(f"fe_{nel}", A, p, np.arange(n), rng.random(n), check_dense_lu=True)
    A = mats.poisson2d(16)
    q = Plan(A).q()
    save("poisson2d_16", A, q, q, rng.random(A.shape[0]))
    A = mats.poisson3d(6)
    q = Plan(A, grid=(6, 6, 6)).q()
    save("poisson3d_6", A, q, q, rng.random(A.shape[0]))
    A = mats.random_dominant(200, 0.02, 47)
    q = Plan(A).q()
    save("random_dominant_200", A, q, q, rng.random(A.shape[0]))
    A = mats.random_dominant(1000, 0.01, 47)    # C1 (BASELINE.json configs[0])
    save_c1("c1_random_1000", A, Plan(A).q(), np.random.default_rng(47).random(1000))


if __name__ == "__main__":
    main()
