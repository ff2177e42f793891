"""Synthetic workloads of BASELINE.json's configs: Kronecker-sum Poisson
matrices and the 1 %-fill random matrix with a dominant diagonal.  Pure scipy; these build
inputs, they compute nothing of the factorization."""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp


def _T(N):
    return sp.diags([-np.ones(N - 1), 2 * np.ones(N), -np.ones(N - 1)], [-1, 0, 1], format="csr")


def poisson2d(N):
    """5-point Laplacian kron(T,I) + kron(I,T) on an N x N grid (vertex i + N*j)."""
    T = _T(N)
    I = sp.identity(N, format="csr")
    return sp.csc_matrix(sp.kron(I, T) + sp.kron(T, I))


def poisson3d(N):
    """7-point Laplacian on an N^3 grid as a Kronecker sum (vertex i + N*(j + N*k)).
    Built directly in CSC to keep memory modest at N = 128."""
    n = N ** 3
    idx = np.arange(n, dtype=np.int64)
    i = idx % N
    j = (idx // N) % N
    k = idx // (N * N)
    rows = [idx]
    cols = [idx]
    vals = [np.full(n, 6.0)]
    for d, coord in ((1, i), (N, j), (N * N, k)):
        m = coord > 0
        rows.append(idx[m]); cols.append(idx[m] - d); vals.append(np.full(m.sum(), -1.0))
        m = coord < N - 1
        rows.append(idx[m]); cols.append(idx[m] + d); vals.append(np.full(m.sum(), -1.0))
    r = np.concatenate(rows); c = np.concatenate(cols); v = np.concatenate(vals)
    A = sp.csc_matrix((v, (r, c)), shape=(n, n))
    A.sort_indices()
    return A


def random_dominant(n=1000, density=0.01, seed=47):
    """C1: Bernoulli(density) off-diagonal pattern with U(0,1) values, diagonal 1 + sum_j |a_ij|
    (strictly row- and column-dominant is not required; rows are)."""
    rng = np.random.default_rng(seed)
    mask = rng.random((n, n)) < density
    np.fill_diagonal(mask, False)
    r, c = np.nonzero(mask)
    v = rng.random(r.size)
    A = sp.csr_matrix((v, (r, c)), shape=(n, n))
    d = 1.0 + np.asarray(abs(A).sum(axis=1)).ravel()
    A = A + sp.diags(d)
    A = sp.csc_matrix(A)
    A.sort_indices()
    return A


def perturb_diag(A, seed):
    """C5: same pattern, new values: diag += U(0,1) from default_rng(seed)."""
    A = sp.csc_matrix(A, copy=True)
    rng = np.random.default_rng(seed)
    n = A.shape[0]
    d = rng.random(n)
    # diagonal positions in CSC
    for j in range(n):
        s, e = A.indptr[j], A.indptr[j + 1]
        rows = A.indices[s:e]
        t = np.searchsorted(rows, j)
        if t < rows.size and rows[t] == j:
            A.data[s + t] += d[j]
    return A


def diag_positions(A):
    """Index into A.data of each diagonal entry (vectorised, for fast refactor inputs)."""
    A = sp.csc_matrix(A)
    n = A.shape[0]
    cols = np.repeat(np.arange(n), np.diff(A.indptr))
    return np.nonzero(A.indices == cols)[0]
