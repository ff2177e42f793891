"""Python mirror of the reference's Julia surface (SharedMemSparseLU.jl, src/SharedMemSparseLU.jl).

Julia name                          here                          reference
----------------------------------  ----------------------------  -----------------------
ParallelSparseLU(A, chunk_size)     ParallelSparseLU(A, cs)       :64-98
lu!(F, A)                           lu_(F, A)                     :245-279
ldiv!(x, F, b)                      ldiv_(x, F, b)                :286-342
lsolve!(F, x), rsolve!(F, x)        lsolve_(F, x), rsolve_(F, x)  :349-392
F.L F.U F.p F.q F.Rs                F.L F.U F.p F.q F.Rs          :45-52 (0-based here)
cleanup_ParallelSparseLU!(F)        cleanup_ParallelSparseLU_(F)  :31 (exported, undefined there)
DimensionMismatch                   DimensionMismatch             :288-290
SingularException (UMFPACK)         SingularException             :74 / :247

Tf = ComplexF64 (the reference is generic in Tf, :43, :64, :286): pass a complex matrix and
complex vectors to the same functions; the library factors the real-equivalent 2n x 2n matrix
(``smlu_create_z``, include/smlu.h), so F.L / F.U / F.p / F.q / F.Rs of a complex F are those
of that real-equivalent matrix (2n rows).

All numerics run on the MI355X through libsmlu.so; nothing here computes factors or solves.
"""
from __future__ import annotations

import ctypes

import numpy as np
import scipy.sparse as sp

from . import _lib as C


class DimensionMismatch(ValueError):
    """Julia's DimensionMismatch (src/SharedMemSparseLU.jl:288-290)."""


class SingularException(np.linalg.LinAlgError):
    """UMFPACK's SingularException raised by lu(A)/lu!(F, A) with check=true."""

    def __init__(self, col):
        super().__init__(f"matrix is singular: zero pivot at column {col}")
        self.info = col


class SmluError(RuntimeError):
    pass


def _csc(A):
    dt = np.complex128 if (np.iscomplexobj(A.data) if sp.issparse(A) else np.iscomplexobj(A)) \
        else np.float64
    if not sp.issparse(A):
        A = sp.csc_matrix(np.asarray(A, dtype=dt))
    A = sp.csc_matrix(A, dtype=dt)
    if not A.has_sorted_indices:
        A = A.sorted_indices()
    A.sum_duplicates()
    return A


def _check(rc, h=None):
    if rc < 0:
        raise SmluError(f"libsmlu error {rc}: {C.last_error(h)}")
    return rc


class ParallelSparseLU:
    """LU factorisation of a square sparse matrix on the MI355X.

    ``F.L * F.U == (F.Rs[:, None] * A)[F.p][:, F.q]`` (UMFPACK's relation quoted at
    src/SharedMemSparseLU.jl:305-316), with 0-based ``p``/``q``.
    """

    def __init__(self, A, chunk_size=None, *, ordering="auto", grid=None, device=0,
                 profile=False, p=None, q=None, Rs=None, pivot_tol=None, diag_pivot_tol=None,
                 leaf_size=None, relax=True, use_mfma=None, refine=None,
                 int32_indices=False, L_pattern=None, U_pattern=None):
        A = _csc(A)
        m, n = A.shape
        if m != n:
            raise DimensionMismatch(f"matrix is not square: {m} x {n}")
        if chunk_size is None:
            chunk_size = 8                       # :67-70
        chunk_size = min(int(chunk_size), n)     # :72
        order = {"auto": C.ORDER_AUTO, "natural": C.ORDER_NATURAL, "nd": C.ORDER_GRAPH_ND,
                 "geometric": C.ORDER_GEOMETRIC_ND, "amd": C.ORDER_AMD, "given": C.ORDER_GIVEN}[ordering]
        kw = dict(chunk_size=chunk_size, index_base=0, ordering=order, device=device,
                  profile=1 if profile else 0, relax=1 if relax else 0)
        if grid is not None:
            kw["grid"] = grid
            if ordering == "auto":
                kw["ordering"] = C.ORDER_GEOMETRIC_ND
        if pivot_tol is not None:
            kw["pivot_tol"] = float(pivot_tol)
        if diag_pivot_tol is not None:
            kw["diag_pivot_tol"] = float(diag_pivot_tol)
        if leaf_size is not None:
            kw["leaf_size"] = int(leaf_size)
        if use_mfma is not None:
            kw["use_mfma"] = 1 if use_mfma else 0
        if refine is not None:
            kw["refine"] = int(refine)
        self._opts = C.default_opts(**kw)
        self.m, self.n = m, n
        self.chunk_size = chunk_size
        self.is_complex = A.dtype == np.complex128
        self._dt = A.dtype
        self._colptr = np.ascontiguousarray(A.indptr, dtype=np.int64)
        self._rowval = np.ascontiguousarray(A.indices, dtype=np.int64)
        vals = np.ascontiguousarray(A.data, dtype=self._dt)
        h = ctypes.c_void_p()
        L = C.lib()
        if self.is_complex:
            if p is not None or q is not None or int32_indices:
                raise ValueError("complex matrices take neither a given (p, q) nor Int32 indices")
            rc = L.smlu_create_z(n, C.ptr(self._colptr), C.ptr(self._rowval), C.ptr(vals),
                                 ctypes.byref(self._opts), ctypes.byref(h))
        elif p is not None or q is not None:
            pp = np.ascontiguousarray(p, dtype=np.int64)
            qq = np.ascontiguousarray(q, dtype=np.int64)
            rs = None if Rs is None else np.ascontiguousarray(Rs, dtype=np.float64)
            # UMFPACK's F.L / F.U patterns: any sparse matrix, only the pattern is used
            pat = []
            for M in (L_pattern, U_pattern):
                if M is None:
                    pat += [None, None]
                else:
                    M = sp.csc_matrix(M)
                    M.sort_indices()
                    pat += [np.ascontiguousarray(M.indptr, dtype=np.int64),
                            np.ascontiguousarray(M.indices, dtype=np.int64)]
            rc = L.smlu_create_with_pivots(n, C.ptr(self._colptr), C.ptr(self._rowval), C.ptr(vals),
                                           C.ptr(pp), C.ptr(qq), C.ptr(rs), *[C.ptr(a) for a in pat],
                                           ctypes.byref(self._opts), ctypes.byref(h))
        elif int32_indices:
            # SparseMatrixCSC{Float64,Int32}: the Int32 entry point
            cp32 = np.ascontiguousarray(A.indptr, dtype=np.int32)
            ri32 = np.ascontiguousarray(A.indices, dtype=np.int32)
            rc = L.smlu_create_i32(n, C.ptr(cp32), C.ptr(ri32), C.ptr(vals),
                                   ctypes.byref(self._opts), ctypes.byref(h))
        else:
            rc = L.smlu_create(n, C.ptr(self._colptr), C.ptr(self._rowval), C.ptr(vals),
                               ctypes.byref(self._opts), ctypes.byref(h))
        if rc < 0:
            raise SmluError(f"smlu_create failed ({rc}): {C.last_error(None)}")
        self._h = h
        self._factors = None
        if rc == C.SMLU_SINGULAR:
            col = L.smlu_last_error_col(h)
            self.close()
            raise SingularException(col)

    # ---- factor access (F.L, F.U, F.p, F.q, F.Rs) ----
    def _download(self):
        """F.L, F.U, F.p, F.q, F.Rs as the reference has them: complex n x n factors on a complex
        handle (smlu_get_factors_z), real ones otherwise."""
        if not self.is_complex:
            return self.real_equivalent_factors()
        if getattr(self, "_zfactors", None) is None:
            L = C.lib()
            n = self.n
            nl, nu = ctypes.c_int64(), ctypes.c_int64()
            _check(L.smlu_get_sizes_z(self._h, None, ctypes.byref(nl), ctypes.byref(nu)), self._h)
            Lp = np.empty(n + 1, np.int64); Li = np.empty(nl.value, np.int64); Lx = np.empty(nl.value, np.complex128)
            Up = np.empty(n + 1, np.int64); Ui = np.empty(nu.value, np.int64); Ux = np.empty(nu.value, np.complex128)
            p = np.empty(n, np.int64); q = np.empty(n, np.int64); Rs = np.empty(n)
            _check(L.smlu_get_factors_z(self._h, C.ptr(Lp), C.ptr(Li), C.ptr(Lx), C.ptr(Up), C.ptr(Ui),
                                        C.ptr(Ux), C.ptr(p), C.ptr(q), C.ptr(Rs)), self._h)
            self._zfactors = dict(L=sp.csc_matrix((Lx, Li, Lp), shape=(n, n)),
                                  U=sp.csc_matrix((Ux, Ui, Up), shape=(n, n)), p=p, q=q, Rs=Rs)
        return self._zfactors

    def real_equivalent_factors(self):
        """The factors the GPU holds: on a complex handle those of the 2n x 2n real-equivalent K."""
        if self._factors is None:
            L = C.lib()
            n = 2 * self.n if self.is_complex else self.n   # complex: the real-equivalent matrix
            nl, nu = ctypes.c_int64(), ctypes.c_int64()
            _check(L.smlu_get_sizes(self._h, None, ctypes.byref(nl), ctypes.byref(nu)), self._h)
            Lp = np.empty(n + 1, np.int64); Li = np.empty(nl.value, np.int64); Lx = np.empty(nl.value)
            Up = np.empty(n + 1, np.int64); Ui = np.empty(nu.value, np.int64); Ux = np.empty(nu.value)
            p = np.empty(n, np.int64); q = np.empty(n, np.int64); Rs = np.empty(n)
            _check(L.smlu_get_factors(self._h, C.ptr(Lp), C.ptr(Li), C.ptr(Lx), C.ptr(Up), C.ptr(Ui),
                                      C.ptr(Ux), C.ptr(p), C.ptr(q), C.ptr(Rs)), self._h)
            self._factors = dict(L=sp.csc_matrix((Lx, Li, Lp), shape=(n, n)),
                                 U=sp.csc_matrix((Ux, Ui, Up), shape=(n, n)), p=p, q=q, Rs=Rs)
        return self._factors

    @property
    def L(self):
        return self._download()["L"]

    @property
    def U(self):
        return self._download()["U"]

    @property
    def p(self):
        return self._download()["p"]

    @property
    def q(self):
        return self._download()["q"]

    @property
    def Rs(self):
        return self._download()["Rs"]

    def stat(self, key):
        return C.lib().smlu_stat(self._h, key.encode())

    def perm_scale(self):
        """(F.p, F.q, F.Rs) without downloading L and U (smlu_get_factors with NULL factor
        pointers); real-equivalent order on a complex handle."""
        n = 2 * self.n if self.is_complex else self.n
        p = np.empty(n, np.int64); q = np.empty(n, np.int64); Rs = np.empty(n)
        _check(C.lib().smlu_get_factors(self._h, None, None, None, None, None, None, C.ptr(p), C.ptr(q),
                                        C.ptr(Rs)), self._h)
        return p, q, Rs

    def front_store(self):
        """Diagnostics (smlu_dev_front_offsets / smlu_dev_copy): the factor store as one host array
        and per front (Loff, Uoff, Foff, M); front s is store[Loff:Loff+M*ns] (L panel, ld M) and
        store[Uoff:Uoff+ns*nu] (U12, ld ns)."""
        L = C.lib()
        ns = int(self.stat("nsuper"))
        off = np.empty(4 * ns, np.int64)
        _check(L.smlu_dev_front_offsets(self._h, C.ptr(off)), self._h)
        ln = ctypes.c_int64()
        _check(L.smlu_dev_copy(self._h, 0, 0, -1, None, ctypes.byref(ln)), self._h)
        store = np.empty(ln.value)
        _check(L.smlu_dev_copy(self._h, 0, 0, ln.value, C.ptr(store), None), self._h)
        return store, off.reshape(ns, 4)

    def fronts(self):
        """The analysis' assembly tree and the current schedule's pivot-candidate mode per front
        (smlu_get_fronts): dict(first, parent, rowptr, rows, p0, mode), 0-based."""
        ns = int(self.stat("nsuper"))
        n = int(self.stat("n"))
        first = np.empty(ns + 1, np.int64)
        parent = np.empty(ns, np.int64)
        rowptr = np.empty(ns + 1, np.int64)
        mode = np.empty(ns, np.int32)
        L = C.lib()
        _check(L.smlu_get_fronts(self._h, C.ptr(first), C.ptr(parent), C.ptr(rowptr), None, None,
                                 C.ptr(mode)), self._h)
        rows = np.empty(rowptr[-1], np.int64)
        p0 = np.empty(n, np.int64)
        _check(L.smlu_get_fronts(self._h, None, None, None, C.ptr(rows), C.ptr(p0), None), self._h)
        return dict(first=first, parent=parent, rowptr=rowptr, rows=rows, p0=p0, mode=mode)

    def refactor(self, values):
        """lu!(F, A) with host values in A's CSC order (same pattern): smlu_refactor, the call the
        Julia shim makes (src/SharedMemSparseLU.jl:245-279)."""
        v = np.ascontiguousarray(values, dtype=self._dt)
        L = C.lib()
        rc = _check((L.smlu_refactor_z if self.is_complex else L.smlu_refactor)(self._h, C.ptr(v)), self._h)
        self._factors = None
        self._zfactors = None
        if rc == C.SMLU_SINGULAR:
            raise SingularException(L.smlu_last_error_col(self._h))
        return rc

    # ---- device-resident entry points (values / vectors already in HBM) ----
    def refactor_device(self, d_values):
        """lu! with values already on the device (torch tensor or raw pointer int; complex
        handles take interleaved complex values, e.g. a complex128 tensor)."""
        ptr = d_values.data_ptr() if hasattr(d_values, "data_ptr") else int(d_values)
        fn = C.lib().smlu_refactor_z_device if self.is_complex else C.lib().smlu_refactor_device
        with C.caller_stream(self._h, d_values):
            rc = _check(fn(self._h, ctypes.c_void_p(ptr)), self._h)
        self._factors = None
        self._zfactors = None
        if rc == C.SMLU_SINGULAR:
            raise SingularException(C.lib().smlu_last_error_col(self._h))
        return rc

    def solve_device(self, d_x, d_b):
        px = d_x.data_ptr() if hasattr(d_x, "data_ptr") else int(d_x)
        pb = d_b.data_ptr() if hasattr(d_b, "data_ptr") else int(d_b)
        with C.caller_stream(self._h, d_b):
            return _check(C.lib().smlu_solve_device(self._h, ctypes.c_void_p(pb), ctypes.c_void_p(px)),
                          self._h)

    def solve_multi_device(self, d_X, d_B):
        """ldiv! for several right-hand sides on the device: d_B, d_X are (nrhs, n) contiguous
        torch tensors (column r = row r, i.e. column-major n x nrhs).  One GPU: batches of up to
        16 columns go through the solve kernels together."""
        nrhs, n = d_B.shape
        if n != self.n or tuple(d_X.shape) != (nrhs, n):
            raise DimensionMismatch(f"B has shape {tuple(d_B.shape)}, X has shape {tuple(d_X.shape)}, n={self.n}")
        ld = 2 * n if self.is_complex else n     # leading dimension in doubles
        with C.caller_stream(self._h, d_B):
            return _check(C.lib().smlu_solve_multi_device(self._h, nrhs, ctypes.c_void_p(d_B.data_ptr()), ld,
                                                          ctypes.c_void_p(d_X.data_ptr()), ld), self._h)

    def close(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            C.lib().smlu_destroy(h)
        self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __repr__(self):
        return f"ParallelSparseLU(n={self.n}, nnz(L+U)={self.stat('nnzLU'):.0f})"


def lu_(F: ParallelSparseLU, A):
    """lu!(F, A) — src/SharedMemSparseLU.jl:245-279.  Same pattern: numeric refactor on the
    GPU; different pattern: re-analysis (the reference's reallocate branch, :252-273)."""
    A = _csc(A)
    if A.shape != (F.m, F.n):
        raise DimensionMismatch(f"A has size {A.shape}, F has size {(F.m, F.n)}")
    if A.dtype == np.complex128 and not F.is_complex:
        raise TypeError("complex values for a real factorization (create it from a complex matrix)")
    vals = np.ascontiguousarray(A.data, dtype=F._dt)   # real values into a complex F are promoted
    L = C.lib()
    same = (A.nnz == F._rowval.size and np.array_equal(A.indptr, F._colptr)
            and np.array_equal(A.indices, F._rowval))
    if same:
        rc = (L.smlu_refactor_z if F.is_complex else L.smlu_refactor)(F._h, C.ptr(vals))
    else:
        F._colptr = np.ascontiguousarray(A.indptr, dtype=np.int64)
        F._rowval = np.ascontiguousarray(A.indices, dtype=np.int64)
        fn = L.smlu_refactor_csc_z if F.is_complex else L.smlu_refactor_csc
        rc = fn(F._h, F.n, C.ptr(F._colptr), C.ptr(F._rowval), C.ptr(vals))
    F._factors = None
    F._zfactors = None
    _check(rc, F._h)
    if rc == C.SMLU_SINGULAR:
        raise SingularException(L.smlu_last_error_col(F._h))
    return None


def ldiv_(x, F: ParallelSparseLU, b):
    """ldiv!(x, F, b) — src/SharedMemSparseLU.jl:286-342.  ``x is b`` is allowed."""
    if F.m != F.n:
        raise DimensionMismatch(f"`F` is not square: F.m={F.m}, F.n={F.n}")
    if len(x) != F.n:
        raise DimensionMismatch(f"`x` does not have same size as F: length(x)={len(x)}, F.n={F.n}")
    if len(b) != F.n:
        raise DimensionMismatch(f"`b` does not have same size as F: length(b)={len(b)}, F.n={F.n}")
    if not F.is_complex and (np.iscomplexobj(b) or np.iscomplexobj(x)):
        raise TypeError("complex vectors need a factorization of a complex matrix")
    _need_complex_x(F, x)
    if np.ndim(b) == 2 or np.ndim(x) == 2:
        # several right-hand sides (columns), SURVEY §8f-4: one C-ABI call, column-major buffers
        if np.shape(x) != np.shape(b):
            raise DimensionMismatch(f"`x` has size {np.shape(x)}, `b` has size {np.shape(b)}")
        nrhs = np.shape(b)[1]
        dt = F._dt
        bb = np.asfortranarray(b, dtype=dt)
        xx = x if (isinstance(x, np.ndarray) and x.dtype == dt and x.flags.f_contiguous) \
            else np.empty((F.n, nrhs), dtype=dt, order="F")
        ld = 2 * F.n if F.is_complex else F.n   # leading dimension in doubles
        _check(C.lib().smlu_solve_multi(F._h, nrhs, C.ptr(bb), ld, C.ptr(xx), ld), F._h)
        if xx is not x:
            x[:, :] = xx
        return x
    bb = np.ascontiguousarray(b, dtype=F._dt)
    xx = x if (isinstance(x, np.ndarray) and x.dtype == F._dt and x.flags.c_contiguous) \
        else np.empty(F.n, dtype=F._dt)
    _check(C.lib().smlu_solve(F._h, C.ptr(bb), C.ptr(xx)), F._h)
    if xx is not x:
        x[:] = xx
    return x


def _need_complex_x(F, x):
    """A complex factorization writes a complex solution: a real x would silently drop the
    imaginary part (Julia raises InexactError there), so it is refused."""
    if F.is_complex and not np.iscomplexobj(x):
        raise TypeError("the solution of a complex factorization needs a complex x")


def _tri(F, x, which):
    _need_complex_x(F, x)
    if len(x) != F.n:
        raise DimensionMismatch(f"`x` does not have same size as F: length(x)={len(x)}, F.n={F.n}")
    xx = x if (isinstance(x, np.ndarray) and x.dtype == F._dt and x.flags.c_contiguous) \
        else np.ascontiguousarray(x, dtype=F._dt)
    fn = C.lib().smlu_lsolve if which == "L" else C.lib().smlu_rsolve
    _check(fn(F._h, C.ptr(xx)), F._h)
    if xx is not x:
        x[:] = xx
    return None


def lsolve_(F: ParallelSparseLU, x):
    """lsolve!(F, x) — src/SharedMemSparseLU.jl:349-367: in place ``L \\ x``."""
    return _tri(F, x, "L")


def rsolve_(F: ParallelSparseLU, x):
    """rsolve!(F, x) — src/SharedMemSparseLU.jl:374-392: in place ``U \\ x``."""
    return _tri(F, x, "U")


def chunked_setup(F: ParallelSparseLU, chunk_size=None):
    """Build the reference's dense-chunk solve layout on the GPU from F's current factors
    (get_chunking_parameters / allocate_chunks / fill_chunks!, src/SharedMemSparseLU.jl:101-243;
    chunk_size defaults to 8 as :67-70).  SURVEY §8f-3 parity mode for small banded systems."""
    _check(C.lib().smlu_chunked_setup(F._h, 0 if chunk_size is None else int(chunk_size)), F._h)


def chunked_ldiv_(x, F: ParallelSparseLU, b):
    """ldiv!(x, F, b) (:286-342) through the chunked layout: lsolve!/rsolve! (:349-392) chunk by
    chunk on the GPU.  Same DimensionMismatch checks as ldiv_; x may be b."""
    if len(x) != F.n or len(b) != F.n:
        raise DimensionMismatch(f"x and b must have length F.n={F.n}: {len(x)}, {len(b)}")
    _need_complex_x(F, x)
    bb = np.ascontiguousarray(b, dtype=F._dt)
    xx = np.empty(F.n, dtype=F._dt)
    _check(C.lib().smlu_chunked_ldiv(F._h, C.ptr(bb), C.ptr(xx)), F._h)
    x[:] = xx
    return x


def cleanup_ParallelSparseLU_(F: ParallelSparseLU):
    """cleanup_ParallelSparseLU!(F) — exported but undefined in the reference (:31); here it
    releases the device memory, stream and host plan of F."""
    F.close()


def allocate_shared(T, *dims):
    """allocate_shared — exported but undefined in the reference (:31).  There are no MPI
    shared-memory windows on the GPU path; this returns a zeroed host array of the shape."""
    return np.zeros(dims, dtype=T)
