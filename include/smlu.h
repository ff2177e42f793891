/*
 * smlu.h — C-ABI of libsmlu.so, the MI355X-native (gfx950) sparse LU refactorize/solve
 * library that is a drop-in for the hot path of SharedMemSparseLU.jl
 * (reference snapshot 2024-10-20, /root/reference).
 *
 * Every entry point below names the reference interface it replaces (file:line in
 * /root/reference).  Plain C types only: int64_t indices, double values, opaque handles.
 *
 * Conventions
 *   - Matrices cross the boundary in CSC form (colptr[n+1], rowval[nnz], nzval[nnz]),
 *     1-based by default (Julia's SparseMatrixCSC{Float64,Int64}); set
 *     smlu_opts.index_base = 0 for 0-based (scipy / C) callers.
 *   - Host arrays are borrowed for the duration of the call only; the library copies
 *     what it needs and owns all device memory and one HIP stream per handle.
 *   - Status: 0 = SMLU_OK; positive = numerical status (singular / weak pivot);
 *     negative = usage, allocation or HIP errors.  smlu_last_error_string() explains.
 *   - Thread-compatible: distinct handles may be used concurrently; calls on one handle
 *     must be serialised (the reference's `wrk` vector is likewise shared per factor,
 *     src/SharedMemSparseLU.jl:318).
 */
#ifndef SMLU_H
#define SMLU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ---------------------------------------------------------------- */
#define SMLU_OK                 0
#define SMLU_SINGULAR           1   /* zero pivot column (UMFPACK SingularException, src/SharedMemSparseLU.jl:74) */
#define SMLU_PIVOT_WEAK         2   /* a pivot failed the threshold test (growth > 1/pivot_tol) */
#define SMLU_ERR_ARG          (-1)  /* bad argument / DimensionMismatch (src/SharedMemSparseLU.jl:288-290) */
#define SMLU_ERR_PATTERN      (-2)  /* refactor called with a different sparsity pattern */
#define SMLU_ERR_ALLOC        (-3)  /* host or device allocation failed */
#define SMLU_ERR_HIP          (-4)  /* HIP runtime error */
#define SMLU_ERR_NODEVICE     (-5)  /* no gfx950 device visible: the library never falls back to the CPU */
#define SMLU_ERR_STATE        (-6)  /* handle has no numeric factorization */

/* ---- ordering choices ------------------------------------------------------------- */
#define SMLU_ORDER_AUTO         0   /* geometric ND if grid[] given, else graph nested dissection */
#define SMLU_ORDER_NATURAL      1
#define SMLU_ORDER_GEOMETRIC_ND 2   /* needs grid[0..2]: vertex v = i + nx*(j + ny*k) */
#define SMLU_ORDER_GRAPH_ND     3   /* BFS level-structure nested dissection on A+A' */
#define SMLU_ORDER_GIVEN        4   /* use smlu_create_with_pivots' p and q unchanged */

typedef struct smlu_opts {
    int64_t chunk_size;   /* reference `chunk_size` (src/SharedMemSparseLU.jl:64-72); accepted, clamped to n */
    int32_t index_base;   /* 1 (Julia, default) or 0 */
    int32_t ordering;     /* SMLU_ORDER_* */
    int64_t grid[3];      /* grid dimensions for SMLU_ORDER_GEOMETRIC_ND (0 = unset) */
    int32_t scale;        /* 1 = UMFPACK SUM row scaling Rs[i] = 1/sum_j |a_ij| (default), 0 = none */
    int32_t relax;        /* 1 = relaxed supernode amalgamation (default) */
    double  pivot_tol;    /* threshold partial pivoting tolerance (UMFPACK default 0.1) */
    double  diag_pivot_tol; /* diagonal preference: keep a_kk unless some candidate exceeds
                               |a_kk|/diag_pivot_tol (default 0.1; UMFPACK's symmetric default 0.001) */
    int32_t device;       /* HIP device ordinal (default 0) */
    int32_t profile;      /* 1 = record per-kernel-class HIP events during refactor/solve */
    int64_t leaf_size;    /* nested-dissection leaf size (default 64) */
    int32_t use_mfma;     /* 1 (default) = fp64 MFMA (v_mfma_f64_16x16x4) for the dense Schur
                             updates of large launches; 0 = fp64 VALU tiles (env SMLU_VALU_GEMM).
                             Bitwise-identical results; MFMA is faster on large tiles */
    int32_t refine;       /* iterative-refinement steps in smlu_solve*: -1 (default) = up to 3 only
                             when the last factorization flagged weak pivots (the pivot-failure
                             fallback of the diagonal-tile pivoting); 0 = never;
                             k > 0 = up to k steps (stops when the residual stops halving) */
} smlu_opts;

typedef struct smlu_handle smlu_handle;

/* Fill `opts` with the defaults listed above. */
void smlu_default_opts(smlu_opts* opts);

/* ParallelSparseLU(A, chunk_size) — src/SharedMemSparseLU.jl:64-98.
 * Host symbolic analysis (ordering, elimination tree, supernodes, level schedule), upload,
 * then the first numeric factorization on the GPU.  Returns SMLU_SINGULAR when A is
 * numerically singular (the reference's UMFPACK `lu(A)` throws SingularException). */
int smlu_create(int64_t n, const int64_t* colptr, const int64_t* rowval, const double* nzval,
                const smlu_opts* opts, smlu_handle** out);

/* As smlu_create, but with the caller's row order p and column order q (1-based or 0-based
 * per opts), and optionally Rs (NULL = compute).  Used by the Julia shim to hand over
 * UMFPACK's own (p, q, Rs) so that pivot order matches the reference by construction
 * (SURVEY §8f-1).  No pivoting is performed on top of the given order. */
int smlu_create_with_pivots(int64_t n, const int64_t* colptr, const int64_t* rowval,
                            const double* nzval, const int64_t* p, const int64_t* q,
                            const double* Rs, const smlu_opts* opts, smlu_handle** out);

/* lu!(F, A) — src/SharedMemSparseLU.jl:245-279: numeric refactorization with the same
 * pattern, new values (nzval in A's original CSC order, host memory). */
int smlu_refactor(smlu_handle* h, const double* nzval);

/* Same, values already resident in device memory (HBM). */
int smlu_refactor_device(smlu_handle* h, const double* d_nzval);

/* lu!(F, A) where A's pattern may differ: re-analyses when it does (the reference's
 * `reallocate` branch, src/SharedMemSparseLU.jl:252-273). */
int smlu_refactor_csc(smlu_handle* h, int64_t n, const int64_t* colptr, const int64_t* rowval,
                      const double* nzval);

/* ldiv!(x, F, b) — src/SharedMemSparseLU.jl:286-342.  Host vectors of length n; x == b allowed. */
int smlu_solve(smlu_handle* h, const double* b, double* x);

/* Same with device pointers (x == b allowed). */
int smlu_solve_device(smlu_handle* h, const double* d_b, double* d_x);

/* r = b - A x with the handle's current A values (device pointers, length n; r may not alias
 * x or b) and its max-norm in *nrm (may be NULL).  The residual step of iterative refinement,
 * exported for callers that drive the partitioned solve (smlu_dist_*). */
int smlu_residual_device(smlu_handle* h, const double* d_x, const double* d_b, double* d_r, double* nrm);

/* ldiv! with nrhs right-hand sides: column j of B (ldb >= n) -> column j of X (ldx >= n),
 * host memory, X == B allowed.  The reference's ldiv! is generic over the vector type
 * (src/SharedMemSparseLU.jl:286); multiple RHS are SURVEY §8f-4. */
int smlu_solve_multi(smlu_handle* h, int64_t nrhs, const double* B, int64_t ldb, double* X, int64_t ldx);

/* Same with device pointers. */
int smlu_solve_multi_device(smlu_handle* h, int64_t nrhs, const double* d_B, int64_t ldb, double* d_X,
                            int64_t ldx);

/* ParallelSparseLU(A::SparseMatrixCSC{Float64,Int32}) — Int32 index arrays;
 * converted to the Int64 path on the host. */
int smlu_create_i32(int64_t n, const int32_t* colptr, const int32_t* rowval, const double* nzval,
                    const smlu_opts* opts, smlu_handle** out);

/* lsolve!(F, x) — src/SharedMemSparseLU.jl:349-367: in place L \ x on an already
 * row-permuted and scaled host vector (x in the reference's F.p order). */
int smlu_lsolve(smlu_handle* h, double* x);

/* rsolve!(F, x) — src/SharedMemSparseLU.jl:374-392: in place U \ x. */
int smlu_rsolve(smlu_handle* h, double* x);

/* The reference's own dense-chunk solve layout on the GPU, a parity mode for
 * small banded systems: chunk geometry, negated rectangles and back-to-front U chunks as
 * get_chunking_parameters / allocate_chunks / fill_chunks! (src/SharedMemSparseLU.jl:101-243)
 * build them from the current factors (chunk_size <= 0: 8, as :67-70; clamped to n, :72).
 * smlu_chunked_ldiv is ldiv! (:286-342) with lsolve!/rsolve! (:349-392) done chunk by chunk
 * (trsv on the diagonal block, then x[rows] += Rect*x[cols]); x may alias b.  The chunks are
 * refilled automatically after a refactor (as lu! does, :265-276).  Refuses (SMLU_ERR_ALLOC)
 * layouts above 32 GB -- the reference's layout is dense and infeasible for large fill. */
int smlu_chunked_setup(smlu_handle* h, int64_t chunk_size);
int smlu_chunked_ldiv(smlu_handle* h, const double* b, double* x);
int smlu_chunked_ldiv_device(smlu_handle* h, const double* d_b, double* d_x);

/* Sizes for smlu_get_factors: n, nnz(L) (incl. unit diagonal), nnz(U). */
int smlu_get_sizes(smlu_handle* h, int64_t* n, int64_t* nnz_L, int64_t* nnz_U);

/* F.L, F.U, F.p, F.q, F.Rs (src/SharedMemSparseLU.jl:45-52; UMFPACK contract
 * F.L*F.U == (F.Rs .* A)[F.p, F.q], quoted at :305-316).  L: CSC, unit diagonal stored
 * first in each column, rows sorted.  U: CSC, rows sorted, diagonal last.  Indices use
 * opts.index_base.  Any pointer may be NULL to skip that output. */
int smlu_get_factors(smlu_handle* h, int64_t* Lcolptr, int64_t* Lrowval, double* Lnzval,
                     int64_t* Ucolptr, int64_t* Urowval, double* Unzval,
                     int64_t* p, int64_t* q, double* Rs);

/* cleanup_ParallelSparseLU!(F) — exported but undefined in the reference
 * (src/SharedMemSparseLU.jl:31): frees device memory, stream and host plan. */
void smlu_destroy(smlu_handle* h);

/* Diagnostics. */
const char* smlu_last_error_string(const smlu_handle* h);   /* h may be NULL: thread-global */
int64_t     smlu_last_error_col(const smlu_handle* h);      /* column of a zero/weak pivot, 0-based, -1 none */

/* Plan statistics (host symbolic analysis): keys are
 * "n","nnzA","nsuper","nlevels","nnzL","nnzU","nnzLU","flops","upd","front_max","ns_max",
 * "factor_bytes","scratch_bytes","launches","analysis_ms","refactor_ms_last","solve_ms_last",
 * "growth_max","dense_flops","gemm_flops","ms_gemm","ms_panel","ms_trsm","ms_assemble",
 * "ms_small","ms_solve". Returns NaN for an unknown key. */
double smlu_stat(const smlu_handle* h, const char* key);

/* ---- host-only symbolic analysis (no GPU needed; used by the CPU test suite) ------- */
typedef struct smlu_plan smlu_plan;
int  smlu_plan_create(int64_t n, const int64_t* colptr, const int64_t* rowval,
                      const smlu_opts* opts, smlu_plan** out);
double smlu_plan_stat(const smlu_plan* plan, const char* key);
/* Column order q (new -> old, 0-based) and the structural pattern of L (CSC, 0-based,
 * unit diagonal first) implied by the plan; NULL pointers are skipped. */
int  smlu_plan_pattern(const smlu_plan* plan, int64_t* q, int64_t* Lcolptr, int64_t* Lrowval);
/* Supernode partition: first column of each supernode (nsuper+1 entries), parent
 * supernode (-1 for roots) and level; NULL pointers are skipped. */
int  smlu_plan_supernodes(const smlu_plan* plan, int64_t* first, int64_t* parent, int64_t* level);
void smlu_plan_destroy(smlu_plan* plan);

/* ---- multi-GPU partition ---------------------------------------------------
 * One process per GPU.  The assembly tree is split by proportional mapping: each rank factors
 * its subtrees with no communication; a front whose child lives on another rank receives that
 * child's update block right before its level ("exchange point").  The library runs the
 * segments between exchange points on its own stream; the caller moves the packed blocks
 * between ranks (RCCL point-to-point over xGMI in the Python mirror, smlu/dist.py).  This
 * replaces the reference's MPI shared-memory column split (src/SharedMemSparseLU.jl:101-160
 * distributes dense chunks over ranks).
 *
 * Factor:  smlu_dist_set_values; for seg in 0..nseg-1: (seg > 0: exchange kind 0 before seg)
 *          smlu_dist_factor_segment(seg).  The last segment returns the pivot status.
 * Solve:   forward  segments (phase 0, exchange kind 1 before seg > 0; seg 0 reads b),
 *          backward segments (phase 1, exchange kind 2 before seg > 0),
 *          phase 2 writes this rank's rows of x (others 0); the caller sums x over ranks.
 * Exchange (kind, seg): smlu_dist_xsizes gives per-peer send/recv counts (doubles);
 *          smlu_dist_pack fills a device buffer with the outgoing blocks in destination-rank
 *          order (kind 2: this rank's rows once, sent to every peer); smlu_dist_unpack takes
 *          the incoming blocks concatenated in source-rank order. */
int     smlu_dist_create(int64_t n, const int64_t* colptr, const int64_t* rowval, const double* nzval,
                         const smlu_opts* opts, int32_t rank, int32_t nranks, smlu_handle** out);
int64_t smlu_dist_nsegments(const smlu_handle* h);
int     smlu_dist_set_values(smlu_handle* h, const double* nzval, int32_t on_device);
int     smlu_dist_factor_segment(smlu_handle* h, int32_t seg);
int     smlu_dist_solve_segment(smlu_handle* h, const double* d_b, double* d_x, int32_t phase, int32_t seg);
int     smlu_dist_xsizes(smlu_handle* h, int32_t kind, int32_t seg, int64_t* send, int64_t* recv);
int     smlu_dist_pack(smlu_handle* h, int32_t kind, int32_t seg, double* d_buf);
int     smlu_dist_unpack(smlu_handle* h, int32_t kind, int32_t seg, const double* d_buf);
/* Host-only: the partition a dist handle of `nparts` ranks would use (owner per supernode,
 * exchange-point levels); NULL outputs are skipped. */
int     smlu_plan_partition(const smlu_plan* plan, int32_t nparts, int32_t* owner, int32_t* xlevels,
                            int64_t* nx);

/* Library version string. */
const char* smlu_version(void);

#ifdef __cplusplus
}
#endif

#endif /* SMLU_H */
