"""CPU oracle for the smlu parity tests.  TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg import
this module, and only as the checker.  The product path (``smlu`` + ``libsmlu.so``) never
imports, links or executes anything under ``oracle/``.

Contents
--------
* ctypes binding of ``liboracle.so`` (oracle.c): UMFPACK-style SUM row scaling, fixed-pivot
  left-looking sparse LU of ``(Rs .* A)[p, q]``, CSC triangular solves and ``ldiv!``
  (reference ``src/SharedMemSparseLU.jl:286-392``).
* :class:`ChunkedSolve` — a verbatim-semantics numpy restatement of the reference's dense
  chunk solve layout: ``get_chunking_parameters`` (:101-149), ``allocate_chunks`` (:151-178),
  ``fill_chunks!`` (:180-243, rectangular chunks store the NEGATED values), ``lsolve!``
  (:349-367, ``trsv!('L','N','U')`` + ``gemm!`` with alpha = beta = 1) and ``rsolve!``
  (:374-392, chunks walked from the back).
* :func:`real_equivalent` — ComplexF64 (the reference is generic in ``Tf``,
  src/SharedMemSparseLU.jl:43,:64,:286): the real 2n x 2n matrix K in which a complex entry
  x + iy is the block [[x, -y], [y, x]] at rows 2i, 2i+1 / columns 2j, 2j+1.  An LU of K is an
  LU of the complex operator; interleaved complex vectors are vectors of K.  The oracle's LU of
  K is the checker of the library's complex path; the complex solutions are pinned against
  scipy's complex SuperLU (tests/test_oracle.py).
* :func:`test_matrix` — the reference's FE-like fixture generator (test/runtests.jl:12-21),
  restated over a numpy Generator (Julia's MersenneTwister stream is not reproduced).

Parity pinning: no reference outputs exist (no Julia, no UMFPACK in this image, nothing
committed in the reference's tests).  The oracle is pinned by (i) the reference's own test
checks restated in tests/test_oracle.py (solution vectors vs. independent solvers at the
reference tolerances 1e-12 / 1e-10, test/runtests.jl:25-26), (ii) the UMFPACK contract
``L*U == (Rs.*A)[p,q]`` (src/SharedMemSparseLU.jl:305-316) and (iii) LAPACK known answers:
with scipy's partial-pivoting row order, the fixed-pivot oracle reproduces scipy.linalg.lu's
L and U.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np
import scipy.linalg as sla
import scipy.sparse as sp

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

_i64p = ctypes.POINTER(ctypes.c_int64)
_f64p = ctypes.POINTER(ctypes.c_double)


def build():
    """Compile liboracle.so (gcc) if missing or stale."""
    so = os.path.join(_HERE, "liboracle.so")
    srcs = [os.path.join(_HERE, f) for f in ("oracle.c", "mf.c", "oracle.h")]
    if not os.path.exists(so) or any(os.path.getmtime(so) < os.path.getmtime(f) for f in srcs):
        subprocess.check_call(["make", "-s", "-C", _HERE])
    return so


def lib():
    global _LIB
    if _LIB is None:
        so = build()
        L = ctypes.CDLL(so)
        L.oracle_rowscale.argtypes = [ctypes.c_int64, _i64p, _i64p, _f64p, _f64p]
        L.oracle_lu_fixed.restype = ctypes.c_void_p
        L.oracle_lu_fixed.argtypes = [ctypes.c_int64, _i64p, _i64p, _f64p, _f64p, _i64p, _i64p,
                                      ctypes.POINTER(ctypes.c_int)]
        L.oracle_lu_free.argtypes = [ctypes.c_void_p]
        L.oracle_lu_nnz.restype = ctypes.c_int64
        L.oracle_lu_nnz.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.oracle_lu_export.argtypes = [ctypes.c_void_p, _i64p, _i64p, _f64p, _i64p, _i64p, _f64p]
        L.oracle_ldiv.argtypes = [ctypes.c_void_p, _f64p, _i64p, _i64p, _f64p, _f64p]
        vp = ctypes.c_void_p
        L.oracle_mf_create.restype = vp
        L.oracle_mf_create.argtypes = [ctypes.c_int64, vp, vp, vp, vp, ctypes.c_int64, vp, vp, vp, vp, vp,
                                       ctypes.c_double, ctypes.c_double, ctypes.c_int,
                                       ctypes.POINTER(ctypes.c_int)]
        L.oracle_mf_set_pairs.argtypes = [vp, ctypes.c_int]
        L.oracle_mf_factor.restype = ctypes.c_int
        L.oracle_mf_factor.argtypes = [vp, vp]
        L.oracle_mf_result.argtypes = [vp, vp, vp, vp]
        L.oracle_mf_destroy.argtypes = [vp]
        L.oracle_mf_front_values.restype = ctypes.c_int64
        L.oracle_mf_front_values.argtypes = [vp, ctypes.c_int64, vp]
        L.oracle_dominant.restype = ctypes.c_int
        L.oracle_dominant.argtypes = [ctypes.c_int64, vp, vp, vp]
        _LIB = L
    return _LIB


def _p(a, t):
    return a.ctypes.data_as(t)


def _csc(A):
    A = sp.csc_matrix(A)
    A.sort_indices()
    A.sum_duplicates()
    return (A, np.ascontiguousarray(A.indptr, dtype=np.int64),
            np.ascontiguousarray(A.indices, dtype=np.int64),
            np.ascontiguousarray(A.data, dtype=np.float64))


def rowscale(A):
    """Rs[i] = 1/sum_j |a_ij| (1 for an empty row) — UMFPACK SUM scaling."""
    A, cp, ri, x = _csc(A)
    n = A.shape[0]
    Rs = np.empty(n)
    lib().oracle_rowscale(n, _p(cp, _i64p), _p(ri, _i64p), _p(x, _f64p), _p(Rs, _f64p))
    return Rs


class OracleLU:
    """Fixed-pivot LU: L*U == (Rs .* A)[p, q] with the given 0-based p, q (new -> old)."""

    def __init__(self, A, p, q, Rs=None):
        A, cp, ri, x = _csc(A)
        n = A.shape[0]
        self.n = n
        self.Rs = np.ascontiguousarray(rowscale(A) if Rs is None else Rs, dtype=np.float64)
        self.p = np.ascontiguousarray(p, dtype=np.int64)
        self.q = np.ascontiguousarray(q, dtype=np.int64)
        st = ctypes.c_int(0)
        h = lib().oracle_lu_fixed(n, _p(cp, _i64p), _p(ri, _i64p), _p(x, _f64p),
                                  _p(self.Rs, _f64p), _p(self.p, _i64p), _p(self.q, _i64p),
                                  ctypes.byref(st))
        if not h:
            raise MemoryError("oracle_lu_fixed failed")
        self.status = st.value
        try:
            nl = lib().oracle_lu_nnz(h, 0)
            nu = lib().oracle_lu_nnz(h, 1)
            Lp = np.empty(n + 1, np.int64); Li = np.empty(nl, np.int64); Lx = np.empty(nl)
            Up = np.empty(n + 1, np.int64); Ui = np.empty(nu, np.int64); Ux = np.empty(nu)
            lib().oracle_lu_export(h, _p(Lp, _i64p), _p(Li, _i64p), _p(Lx, _f64p),
                                   _p(Up, _i64p), _p(Ui, _i64p), _p(Ux, _f64p))
        finally:
            lib().oracle_lu_free(h)
        self.L = sp.csc_matrix((Lx, Li, Lp), shape=(n, n))
        self.U = sp.csc_matrix((Ux, Ui, Up), shape=(n, n))

    def lsolve(self, x):
        """In-place L \\ x (reference lsolve!, src/SharedMemSparseLU.jl:349)."""
        x[:] = _csc_lsolve(self.L, x)
        return x

    def rsolve(self, x):
        """In-place U \\ x (reference rsolve!, src/SharedMemSparseLU.jl:374)."""
        x[:] = _csc_rsolve(self.U, x)
        return x

    def ldiv(self, x, b):
        """ldiv!(x, F, b) (src/SharedMemSparseLU.jl:286-342); x may be b."""
        wrk = self.Rs[self.p] * b[self.p]
        wrk = _csc_lsolve(self.L, wrk)
        wrk = _csc_rsolve(self.U, wrk)
        x[self.q] = wrk
        return x


# --------------------------------------------------------------------------------------
# Independent pivot choice: multifrontal restatement of the GPU's documented pivot rule (mf.c)
# --------------------------------------------------------------------------------------
def _vp(a):
    return None if a is None else ctypes.c_void_p(a.ctypes.data)


def dominant(A):
    """Diagonal dominance by columns or rows (the pivoting-mode test)."""
    A, cp, ri, x = _csc(A)
    return bool(lib().oracle_dominant(A.shape[0], _vp(cp), _vp(ri), _vp(x)))


class MultifrontalOracle:
    """Multifrontal LU of (Rs .* A)[p0, q] over a given assembly tree (mf.c), choosing its own
    pivots with threshold partial pivoting (diagonal preference) inside each front's candidate
    rows.  `fronts`: dict(first, parent, rowptr, rows, p0) as exported by smlu_get_fronts /
    smlu_plan_fronts plus the column order `q`; `mode`: candidate set per front (None: every
    fully-summed row).  factor(values) -> status (0 ok, 1 zero candidate column)."""

    def __init__(self, A, q, fronts, mode=None, diag_tol=0.001, pivot_tol=0.1, threads=1, pairs=False):
        A, cp, ri, _ = _csc(A)
        self.n = A.shape[0]
        self._keep = [np.ascontiguousarray(v, dtype=np.int64) for v in
                      (cp, ri, fronts["p0"], q, fronts["first"], fronts["parent"], fronts["rowptr"],
                       fronts["rows"])]
        cp, ri, p0, q, first, parent, rowptr, rows = self._keep
        self.p0, self.first = p0, first
        self.nsup = first.size - 1
        self.mode = None if mode is None else np.ascontiguousarray(mode, dtype=np.int32)
        st = ctypes.c_int(0)
        self._h = lib().oracle_mf_create(self.n, _vp(cp), _vp(ri), _vp(p0), _vp(q), self.nsup, _vp(first),
                                         _vp(parent), _vp(rowptr), _vp(rows), _vp(self.mode),
                                         float(diag_tol), float(pivot_tol), int(threads), ctypes.byref(st))
        if not self._h:
            raise RuntimeError(f"oracle_mf_create failed ({st.value})")
        if pairs:   # ComplexF64 real-equivalent: pair-preserving pivots (mf.c)
            lib().oracle_mf_set_pairs(self._h, 1)

    def factor(self, values):
        v = np.ascontiguousarray(values, dtype=np.float64)
        rc = lib().oracle_mf_factor(self._h, _vp(v))
        if rc < 0:
            raise MemoryError("oracle_mf_factor failed")
        self.rowperm = np.empty(self.n, np.int32)
        self.flags = np.empty(self.nsup, np.int32)
        self.Rs = np.empty(self.n)
        lib().oracle_mf_result(self._h, _vp(self.rowperm), _vp(self.flags), _vp(self.Rs))
        return rc

    def front_values(self, s):
        """Front s's stored factor values after factor(): L panel (M x ns, ld M) then U12 (ns x nu,
        ld ns), the layout of the GPU's smlu_dev_front_values."""
        cnt = lib().oracle_mf_front_values(self._h, int(s), None)
        if cnt < 0:
            raise IndexError(s)
        out = np.empty(cnt)
        lib().oracle_mf_front_values(self._h, int(s), _vp(out))
        return out

    @property
    def p(self):
        """Final row order: p[k] = p0[first_s + rowperm[k]] (new -> old)."""
        f = np.repeat(self.first[:-1], np.diff(self.first))
        return self.p0[f + self.rowperm]

    def close(self):
        if getattr(self, "_h", None):
            lib().oracle_mf_destroy(self._h)
        self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


SMALL_M = 128        # fronts up to this order are factored whole (mode 0)
FULL_PIV_NS = 512    # blocked fronts with at most this many pivots search every fully-summed row


def front_modes(fronts, pivmode, dominant_values, full_piv_ns=None):
    """The GPU schedule's candidate set per front (restated from DESIGN.md §4 / build_schedule):
    M <= 128 -> 0 (small front, all fully-summed rows); else ns <= limit -> 1 (all fully-summed
    rows), otherwise 2 (the 64 x 64 diagonal tile).  limit: unbounded after a re-pivoting refactor
    (pivmode 1), 0 for dominant values (every blocked front on the diagonal tile), 512 otherwise."""
    first, rowptr = fronts["first"], fronts["rowptr"]
    ns = np.diff(first)
    M = ns + np.diff(rowptr)
    if full_piv_ns is None:
        full_piv_ns = np.iinfo(np.int64).max if pivmode == 1 else (0 if dominant_values else FULL_PIV_NS)
    return np.where(M <= SMALL_M, 0, np.where(ns <= full_piv_ns, 1, 2)).astype(np.int32)


def gpu_pivot_choice(A, q, fronts, *, pivmode=0, dominant_values=None, given=False, pivot_tol=0.1,
                     diag_tol=0.001, full_piv_ns=None, values=None, pairs=False, threads=1, keep=False):
    """Independent restatement of the GPU path's whole pivot decision for one factorization:
    the candidate modes, threshold partial pivoting inside every front (mf.c), and the
    re-pivoting refactor (a zero or weak pivot while diagonal-tile fronts exist -> every blocked
    front again with all fully-summed rows as candidates).  `pivmode`: the handle's mode before
    this factorization (dominant values reset it to 0).  A given (p, q) keeps the diagonal unless
    it is exactly zero (diag_tol 0) and is never re-pivoted.  Returns (p, pivmode, modes, flags),
    and with keep=True also the factored MultifrontalOracle (its front_values; the caller closes it)."""
    A = sp.csc_matrix(A)
    A.sort_indices()
    vals = A.data if values is None else values
    matched = not np.array_equal(fronts["p0"], q)
    if dominant_values is None:
        dominant_values = (not matched and not given) and dominant(sp.csc_matrix((vals, A.indices, A.indptr),
                                                                                 shape=A.shape))
    if dominant_values:
        pivmode = 0
    if pairs:   # a ComplexF64 handle pivots pairs over every fully-summed row of every front
        full_piv_ns = np.iinfo(np.int64).max
    dt = 0.0 if given else diag_tol

    def run(pm):
        modes = front_modes(fronts, pm, dominant_values, full_piv_ns)
        mf = MultifrontalOracle(A, q, fronts, modes, diag_tol=dt, pivot_tol=pivot_tol, pairs=pairs,
                                threads=threads)
        st = mf.factor(vals)
        return mf.p, modes, mf.flags.copy(), st, mf

    p, modes, flags, st, mf = run(pivmode)
    if ((st == 1 or (flags & 2).any()) and pivmode == 0 and (modes == 2).any() and pivot_tol > 0
            and not given and not pairs):
        mf.close()
        pivmode = 1
        p, modes, flags, st, mf = run(1)
    if keep:
        return p, pivmode, modes, flags, mf
    mf.close()
    return p, pivmode, modes, flags


def _csc_lsolve(L, b):
    x = np.array(b, dtype=np.float64, copy=True)
    Lp, Li, Lx = L.indptr, L.indices, L.data
    for j in range(L.shape[0]):
        s, e = Lp[j], Lp[j + 1]
        rows = Li[s:e]
        m = rows != j
        x[rows[m]] -= Lx[s:e][m] * x[j]
    return x


def _csc_rsolve(U, b):
    x = np.array(b, dtype=np.float64, copy=True)
    Up, Ui, Ux = U.indptr, U.indices, U.data
    for j in range(U.shape[0] - 1, -1, -1):
        s, e = Up[j], Up[j + 1]
        x[j] /= Ux[e - 1]
        x[Ui[s:e - 1]] -= Ux[s:e - 1] * x[j]
    return x


# --------------------------------------------------------------------------------------
# Verbatim-semantics restatement of the reference's chunked solve (small n only)
# --------------------------------------------------------------------------------------
class ChunkedSolve:
    """Dense-chunk blocked triangular solves exactly as the reference lays them out.

    L, U: scipy CSC factors following UMFPACK's conventions (L: unit diagonal stored first,
    max row last in each column; U: min row first, diagonal last).  Indices here are 0-based;
    the reference's 1-based ranges are shifted by one.
    """

    def __init__(self, L, U, chunk_size=None):
        L = sp.csc_matrix(L); U = sp.csc_matrix(U)
        L.sort_indices(); U.sort_indices()
        m = L.shape[0]
        n = U.shape[1]
        cs = 8 if chunk_size is None else chunk_size      # :67-70
        cs = min(cs, n)                                   # :72 (clamped with A.n)
        self.m, self.n, self.chunk_size = m, n, cs
        self.total_chunks = (m + cs - 1) // cs            # :108 (uses m, quirk Q1)
        T = self.total_chunks
        self.lcols, self.lrows, self.ucols, self.urows = [], [], [], []
        for chunk in range(1, T + 1):                     # :111-123
            colmin = (chunk - 1) * cs + 1
            colmax = min(m, chunk * cs)
            # maximum(L_rowval[L_colptr[j+1]-1] for j in cols): last (= max) row, 1-based
            rmax = max(L.indices[L.indptr[j + 1] - 1] + 1 for j in range(colmin - 1, colmax))
            self.lcols.append((colmin, colmax))
            self.lrows.append((colmax + 1, rmax))
        for chunk in range(1, T + 1):                     # :132-144 (from the back, Q2)
            colmin = (T - chunk) * cs + 1
            colmax = min(m, (T - chunk + 1) * cs)
            rmin = min(U.indices[U.indptr[j]] + 1 for j in range(colmin - 1, colmax))
            self.ucols.append((colmin, colmax))
            self.urows.append((rmin, colmin - 1))
        # allocate_chunks (:151-178) + fill_chunks! (:180-243)
        self.Lchunks, self.Uchunks = [], []
        for c in range(T):
            cmin, cmax = self.lcols[c]
            rmin, rmax = self.lrows[c]
            tri = np.zeros((cmax - cmin + 1, cmax - cmin + 1))
            rect = np.zeros((max(rmax - rmin + 1, 0), cmax - cmin + 1))
            for col in range(cmin, cmax + 1):
                for jj in range(L.indptr[col - 1], L.indptr[col]):
                    row = L.indices[jj] + 1
                    if row <= cmax:
                        tri[row - cmin, col - cmin] = L.data[jj]
                    else:
                        rect[row - rmin, col - cmin] = -L.data[jj]      # negated (:207, Q3)
            self.Lchunks += [tri, rect]
        for c in range(T):
            cmin, cmax = self.ucols[c]
            rmin, rmax = self.urows[c]
            tri = np.zeros((cmax - cmin + 1, cmax - cmin + 1))
            rect = np.zeros((max(rmax - rmin + 1, 0), cmax - cmin + 1))
            for col in range(cmin, cmax + 1):
                for jj in range(U.indptr[col - 1], U.indptr[col]):
                    row = U.indices[jj] + 1
                    if row >= cmin:
                        tri[row - cmin, col - cmin] = U.data[jj]
                    else:
                        rect[row - rmin, col - cmin] = -U.data[jj]      # negated (:238, Q3)
            self.Uchunks += [tri, rect]

    def lsolve(self, x):
        """lsolve! (:349-367): trsv!('L','N','U') on the diagonal chunk, then gemm! into rows."""
        for c in range(self.total_chunks):
            cmin, cmax = self.lcols[c]
            rmin, rmax = self.lrows[c]
            xs = x[cmin - 1:cmax]
            xs[:] = sla.solve_triangular(self.Lchunks[2 * c], xs, lower=True, unit_diagonal=True)
            if rmax >= rmin:
                x[rmin - 1:rmax] += self.Lchunks[2 * c + 1] @ xs
        return x

    def rsolve(self, x):
        """rsolve! (:374-392): chunks from the back, trsv!('U','N','N') then gemm!."""
        for c in range(self.total_chunks):
            cmin, cmax = self.ucols[c]
            rmin, rmax = self.urows[c]
            xs = x[cmin - 1:cmax]
            xs[:] = sla.solve_triangular(self.Uchunks[2 * c], xs, lower=False)
            if rmax >= rmin:
                x[rmin - 1:rmax] += self.Uchunks[2 * c + 1] @ xs
        return x


# --------------------------------------------------------------------------------------
# Reference fixtures
# --------------------------------------------------------------------------------------
def test_matrix(rng, nel=6, ngr=5):
    """test/runtests.jl:12-21: element blocks written with `.=` (assignment, later elements
    overwrite shared corners), n = nel*(ngr-1)+1."""
    n = nel * (ngr - 1) + 1
    mat = np.zeros((n, n))
    for iel in range(1, nel + 1):
        imin = (iel - 1) * (ngr - 1) + 1
        imax = iel * (ngr - 1) + 1
        mat[imin - 1:imax, imin - 1:imax] = rng.random((ngr, ngr))
    return sp.csc_matrix(mat)


def real_equivalent(A):
    """ComplexF64 A (n x n) -> its real-equivalent K (2n x 2n CSC, sorted): entry a_ij = x + iy
    becomes K[2i, 2j] = x, K[2i+1, 2j] = y, K[2i, 2j+1] = -y, K[2i+1, 2j+1] = x.  Every stored
    complex entry gives four stored entries (zeros included), so K's pattern is value-independent.
    Interleaved complex vectors (re, im, ...) -- ``z.view(np.float64)`` -- are vectors of K."""
    A = sp.csc_matrix(A, dtype=np.complex128)
    A.sort_indices()
    n = A.shape[0]
    cp, ri = A.indptr.astype(np.int64), A.indices.astype(np.int64)
    nnz = cp[-1]
    Kp = np.zeros(2 * n + 1, np.int64)
    Ki = np.empty(4 * nnz, np.int64)
    Kx = np.empty(4 * nnz)
    for j in range(n):
        c0, c = cp[j], cp[j + 1] - cp[j]
        k0 = 4 * c0
        Kp[2 * j + 1] = k0 + 2 * c
        Kp[2 * j + 2] = k0 + 4 * c
        r = ri[c0:c0 + c]
        v = A.data[c0:c0 + c]
        Ki[k0:k0 + 2 * c:2] = 2 * r
        Ki[k0 + 1:k0 + 2 * c:2] = 2 * r + 1
        Kx[k0:k0 + 2 * c:2] = v.real
        Kx[k0 + 1:k0 + 2 * c:2] = v.imag
        Ki[k0 + 2 * c:k0 + 4 * c:2] = 2 * r
        Ki[k0 + 2 * c + 1:k0 + 4 * c:2] = 2 * r + 1
        Kx[k0 + 2 * c:k0 + 4 * c:2] = -v.imag
        Kx[k0 + 2 * c + 1:k0 + 4 * c:2] = v.real
    return sp.csc_matrix((Kx, Ki, Kp), shape=(2 * n, 2 * n))
