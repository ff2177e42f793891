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
/* libsmlu.so is built with -fvisibility=hidden: exactly the functions declared here are exported */
#if defined(__GNUC__)
#pragma GCC visibility push(default)
#endif

/* ---- status codes ---------------------------------------------------------------- */
#define SMLU_OK                 0
#define SMLU_SINGULAR           1   /* zero pivot column (UMFPACK SingularException, src/SharedMemSparseLU.jl:74) */
#define SMLU_PIVOT_WEAK         2   /* a pivot failed the threshold test (growth > 1/pivot_tol) */
#define SMLU_ERR_ARG          (-1)  /* bad argument / DimensionMismatch (src/SharedMemSparseLU.jl:288-290) */
#define SMLU_ERR_PATTERN      (-2)  /* refactor called with a different sparsity pattern, or a given L/U
                                       pattern outside the structural fill of (Rs.*A)[p,q] */
#define SMLU_ERR_ALLOC        (-3)  /* host or device allocation failed */
#define SMLU_ERR_HIP          (-4)  /* HIP runtime error */
#define SMLU_ERR_NODEVICE     (-5)  /* no gfx950 device visible: the library never falls back to the CPU */
#define SMLU_ERR_STATE        (-6)  /* handle has no numeric factorization / illegal device status */

/* ---- ordering choices ------------------------------------------------------------- */
#define SMLU_ORDER_AUTO         0   /* geometric ND if grid[] given, else graph nested dissection */
#define SMLU_ORDER_NATURAL      1
#define SMLU_ORDER_GEOMETRIC_ND 2   /* needs grid[0..2]: vertex v = i + nx*(j + ny*k) */
#define SMLU_ORDER_GRAPH_ND     3   /* BFS level-structure nested dissection on A+A' */
#define SMLU_ORDER_GIVEN        4   /* use smlu_create_with_pivots' p and q unchanged */
#define SMLU_ORDER_AMD          5   /* approximate minimum degree on A+A' (UMFPACK's symmetric-strategy kind) */

typedef struct smlu_opts {
    int64_t chunk_size;   /* reference `chunk_size` (src/SharedMemSparseLU.jl:64-72); accepted, clamped to n */
    int32_t index_base;   /* 1 (Julia, default) or 0 */
    int32_t ordering;     /* SMLU_ORDER_* */
    int64_t grid[3];      /* grid dimensions for SMLU_ORDER_GEOMETRIC_ND (0 = unset) */
    int32_t scale;        /* 1 = UMFPACK SUM row scaling Rs[i] = 1/sum_j |a_ij| (default), 0 = none */
    int32_t relax;        /* 1 = relaxed supernode amalgamation (default) */
    double  pivot_tol;    /* threshold partial pivoting tolerance (UMFPACK default 0.1) */
    double  diag_pivot_tol; /* diagonal preference: keep a_kk when |a_kk| >= diag_pivot_tol times the
                               largest candidate (default 0.001 = UMFPACK's symmetric-strategy
                               SYM_PIVOT_TOLERANCE); otherwise the largest candidate is taken */
    int32_t device;       /* HIP device ordinal (default 0) */
    int32_t profile;      /* 1 = record per-kernel-class HIP events during refactor/solve */
    int64_t leaf_size;    /* nested-dissection leaf size (default 64) */
    int32_t use_mfma;     /* 1 (default) = fp64 MFMA (v_mfma_f64_16x16x4) for the dense Schur
                             updates and the GEMM-form triangular solves; 0 = a comparison path:
                             the VALU 64x64 tile for k > 64 launches and k_step_trsm for the
                             triangular solves (results equal to rounding) */
    int32_t refine;       /* iterative-refinement steps in smlu_solve*: -1 (default) = up to 3 only
                             when the last factorization flagged weak pivots (the pivot-failure
                             fallback of the diagonal-tile pivoting); 0 = never;
                             k > 0 = up to k steps (LAPACK dgerfs' stop: componentwise backward error
                             <= 4 unit roundoffs or not halving) */
    int32_t vendor_gemm;  /* reserved, ignored (round 5 removed the vendor GEMM comparison path:
                             every GEMM runs on the hand-written MFMA tiles) */
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
 * per opts), optionally Rs (NULL = compute) and optionally the L and U patterns (CSC colptr /
 * rowval; L with its unit diagonal first in each column, U with its diagonal last, rows
 * increasing; all four NULL = none).  Used by the Julia shim to hand over UMFPACK's own analysis
 * -- lu(A) and F.p, F.q, F.Rs, F.L, F.U, src/SharedMemSparseLU.jl:74-77, :93-94 -- so that pivot
 * order and L/U pattern match the reference by construction.  No pivoting
 * is performed on top of the given order.  A given pattern must lie inside the structural fill of
 * (Rs.*A)[p, q] (UMFPACK's may miss fill entries that came out exactly zero; smlu_stat
 * "pattern_dropped" counts them), else SMLU_ERR_PATTERN and no handle; smlu_get_factors then
 * exports exactly that pattern. */
int smlu_create_with_pivots(int64_t n, const int64_t* colptr, const int64_t* rowval,
                            const double* nzval, const int64_t* p, const int64_t* q,
                            const double* Rs, const int64_t* Lcolptr, const int64_t* Lrowval,
                            const int64_t* Ucolptr, const int64_t* Urowval, const smlu_opts* opts,
                            smlu_handle** out);

/* lu!(F, A) — src/SharedMemSparseLU.jl:245-279: numeric refactorization with the same
 * pattern, new values (nzval in A's original CSC order, host memory). */
int smlu_refactor(smlu_handle* h, const double* nzval);

/* Same, values already resident in device memory (HBM).  The pivoting mode is re-decided on the
 * new values (a dominance reduction on the device, read back with one stream synchronisation;
 * on a partitioned handle the ranks agree on it through the transport's allreduce). */
int smlu_refactor_device(smlu_handle* h, const double* d_nzval);

/* The caller's stream (a hipStream_t; NULL = the null stream, the default): every *_device
 * entry point orders its reads of caller memory after the work enqueued on that stream so far
 * (an event wait on the handle's stream, no host synchronisation), and returns with its outputs
 * complete.  Set it to the stream that produces the values / right-hand sides (the Python mirror
 * passes torch's current stream on every device call and resets it to NULL afterwards).
 * Lifetime: the handle keeps the raw stream until the next smlu_set_stream; the caller must
 * reset it (NULL) before destroying that stream.  No reference counterpart: Julia's arrays are
 * host memory. */
int smlu_set_stream(smlu_handle* h, void* stream);

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

/* ParallelSparseLU(A::SparseMatrixCSC{ComplexF64}) — the reference is generic in Tf
 * (src/SharedMemSparseLU.jl:43, :64, :286).  nzval holds 2*nnz doubles,
 * interleaved (re, im) per entry (Julia's ComplexF64 / C99 double complex layout).
 * The handle factors the real-equivalent K (2n x 2n, entry x+iy -> block [[x,-y],[y,x]] at rows
 * 2i,2i+1 / columns 2j,2j+1) on the real GPU path, so on a complex handle:
 *   - smlu_solve[_device], smlu_solve_multi[_device], smlu_residual_device, smlu_lsolve/rsolve
 *     and smlu_chunked_* take complex vectors as 2n interleaved doubles (ldb/ldx in doubles);
 *   - smlu_get_sizes / smlu_get_factors describe K's factors (n reported as 2n);
 *   - smlu_last_error_col reports the complex column;  smlu_stat(h, "complex") == 1.
 * The column order is computed on the complex pattern (opts.ordering; SMLU_ORDER_GIVEN is
 * refused) and kept pairwise, so each 2x2 block stays in one front. */
int smlu_create_z(int64_t n, const int64_t* colptr, const int64_t* rowval, const double* nzval,
                  const smlu_opts* opts, smlu_handle** out);

/* lu!(F, A) for a complex handle (same pattern; host values, 2*nnz doubles interleaved). */
int smlu_refactor_z(smlu_handle* h, const double* nzval);

/* Same, complex values already in device memory (16-byte aligned); expanded into K on the GPU. */
int smlu_refactor_z_device(smlu_handle* h, const double* d_nzval);

/* lu!(F, A) for a complex handle where the pattern may differ (re-analysis, :252-273). */
int smlu_refactor_csc_z(smlu_handle* h, int64_t n, const int64_t* colptr, const int64_t* rowval,
                        const double* nzval);

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

/* The assembly tree of the handle's analysis (diagnostic: the tests' pivot-rule oracle replays
 * the GPU's pivot decisions on it).  first[nsup+1]: first column (pivot position) of each front;
 * parent[nsup] (-1: root; parents follow their children); rowptr[nsup+1] / rows[rowptr[nsup]]:
 * the update rows of each front (sorted positions); p0[n]: the row order before pivoting (new ->
 * old, 0-based: q, or q composed with the zero-free-diagonal transversal); mode[nsup]: pivot
 * candidates of the current schedule (0: small front, every fully-summed row; 1: blocked front,
 * every fully-summed row; 2: blocked front, the rows of the 64 x 64 diagonal tile).  The final row
 * order is p[k] = p0[first[s] + rowperm_s[k - first[s]]] for the pivot sequence chosen per front.
 * nsup = smlu_stat(h, "nsuper"); NULL pointers are skipped. */
int smlu_get_fronts(smlu_handle* h, int64_t* first, int64_t* parent, int64_t* rowptr, int64_t* rows,
                    int64_t* p0, int32_t* mode);

/* F.L, F.U, F.p, F.q, F.Rs of a ComplexF64 handle (src/SharedMemSparseLU.jl:47-52: L and U are
 * SparseMatrixCSC{ComplexF64}): the complex n x n factors, values as interleaved (re, im) doubles
 * (2*nnz), same conventions as smlu_get_factors (L unit diagonal first, U diagonal last, rows
 * sorted; F.L*F.U == (F.Rs .* A)[F.p, F.q]).  Folded from the real-equivalent factors: a complex
 * handle pivots K pair by pair (rows 2i, 2i+1 stay adjacent; the diagonal pair is kept when its
 * complex magnitude passes diag_pivot_tol, else the largest pair; inside a pair the larger entry
 * leads, a swap that folds back as a row rotation by -i), so the complex factors always exist
 * (SMLU_ERR_STATE only if a zero-free-diagonal row transversal was needed, which breaks pairs). */
int smlu_get_sizes_z(smlu_handle* h, int64_t* n, int64_t* nnz_L, int64_t* nnz_U);
int smlu_get_factors_z(smlu_handle* h, int64_t* Lcolptr, int64_t* Lrowval, double* Lnzval,
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
/* Update rows of every front (rowptr[nsup+1], rows[rowptr[nsup]], sorted positions) and the
 * row pre-order p0 (new -> old) of a host-only plan; NULL pointers are skipped. */
int  smlu_plan_fronts(const smlu_plan* plan, int64_t* rowptr, int64_t* rows, int64_t* p0);
void smlu_plan_destroy(smlu_plan* plan);

/* ---- multi-GPU partition ---------------------------------------------------
 * One process per GPU; every rank calls the same functions with the same matrix (collective).
 * The assembly tree is split by proportional mapping (each subtree set gets a contiguous rank
 * range sized by a cost model; sibling subtrees get disjoint ranges, so their shared fronts run
 * concurrently); a subtree on one rank is factored with no communication; each front above them
 * is shared by its range as a 1D block-cyclic column partition (blocks of 384 columns): the owner of a pivot
 * block factors it and broadcasts it (L block, pivots, tile inverses) to the group, every
 * member updates the column blocks it owns; the children's F22 columns move to the owners of
 * the parent's columns before its assembly.  Each rank allocates only its own fronts and
 * blocks.  Solves run the same partition (vector segments passed along the block owners, the
 * solution rows of each level shared); x comes out complete on every rank.  This replaces the
 * reference's MPI shared-memory column split (src/SharedMemSparseLU.jl:101-160, the rank split
 * intended at :107, :128).
 *
 * After creation a partitioned handle takes the ordinary entry points (smlu_refactor[_device],
 * smlu_solve[_device], smlu_solve_multi*, smlu_stat); all ranks must call them together.
 * smlu_get_factors, the chunked layout and smlu_refactor_csc are single-GPU only. */

/* Transport between the ranks, supplied by the caller (or the built-in RCCL one below).
 * device_memory = 1: buffers are device pointers ordered on `stream` (a hipStream_t), the
 * callbacks enqueue and return (RCCL); 0: host buffers, the library has synchronised its stream
 * and waits for the callback to complete (host-staged transports such as gloo / MPI).
 * exchange: for each of the npeer peers, send sbytes[i] bytes from sbuf[i] to peer[i] and
 *   receive rbytes[i] bytes from it into rbuf[i] (either may be 0); all must complete.
 * bcast: `bytes` from rank `root` to every rank of `group` (sorted, includes root).
 * allreduce_max: element-wise max of count doubles over all ranks (host memory).
 * Return 0 on success. */
typedef struct smlu_transport {
    void*   ctx;
    int32_t device_memory;
    int (*exchange)(void* ctx, int32_t npeer, const int32_t* peer, void* const* sbuf,
                    const int64_t* sbytes, void* const* rbuf, const int64_t* rbytes, void* stream);
    int (*bcast)(void* ctx, void* buf, int64_t bytes, int32_t root, int32_t gsize,
                 const int32_t* group, void* stream);
    int (*allreduce_max)(void* ctx, double* buf, int32_t count);
} smlu_transport;

/* ParallelSparseLU(A) on `nranks` GPUs (collective): analysis, this rank's allocation, the
 * first factorization.  `tr` is copied; its ctx must stay valid for the handle's life. */
int smlu_dist_create(int64_t n, const int64_t* colptr, const int64_t* rowval, const double* nzval,
                     const smlu_opts* opts, int32_t rank, int32_t nranks, const smlu_transport* tr,
                     smlu_handle** out);

/* Built-in transport over RCCL (xGMI point-to-point): rank 0 calls smlu_rccl_unique_id and
 * shares the 128 bytes with the other ranks (MPI_Bcast in the Julia shim, torch.distributed in
 * the Python mirror); every rank then calls smlu_dist_create_rccl. */
int smlu_rccl_unique_id(uint8_t id[128]);
int smlu_dist_create_rccl(int64_t n, const int64_t* colptr, const int64_t* rowval, const double* nzval,
                          const smlu_opts* opts, int32_t rank, int32_t nranks, const uint8_t id[128],
                          smlu_handle** out);

/* Host-only: the partition a handle of `nparts` ranks would use.  owner[s] = rank of front s,
 * -1 for a front shared by several ranks (its column blocks dealt over its group). */
int     smlu_plan_partition(const smlu_plan* plan, int32_t nparts, int32_t* owner, int64_t* nshared);
/* Host-only: device bytes rank `rank` of `nparts` allocates (factor store, scratch arena,
 * broadcast staging). */
int     smlu_plan_rank_memory(const smlu_plan* plan, int32_t nparts, int32_t rank, double* store_bytes,
                              double* scratch_bytes, double* stage_bytes);
/* Host-only: rank `rank`'s whole schedule of a `nparts`-rank handle, built by the same code as
 * smlu_dist_create but with no device (the pairing check of the collective schedule, e.g. 256^3
 * on 8 ranks in a CPU test).  Its communication steps in execution order, flattened into `ops`
 * (int64 words; ops = NULL: only *len): per step
 *   seq (0 factor, 1 forward solve, 2 backward solve), type (0 exchange, 1 broadcast), root, bytes, cnt,
 *   then cnt x (peer, sbytes, rbytes) for an exchange, or the cnt ranks of the group for a broadcast.
 * bytes[0..4]: device bytes the rank allocates in all, its factor store, its front scratch, its
 * staging + received-block buffer, and the pinned host staging of a host-memory transport; counts[0..2]:
 * factor launches, shared fronts the rank works on, owned column blocks. */
int     smlu_plan_rank_schedule(const smlu_plan* plan, int32_t nparts, int32_t rank, int64_t* ops, int64_t cap,
                                int64_t* len, double bytes[5], int64_t counts[3]);
/* Host-only critical-path projection of the partitioned factorization at `tflops` per GPU,
 * `gbs` GB/s per link and `lat_us` per message: returns the projected seconds, *t1 = one GPU. */
double  smlu_plan_project(const smlu_plan* plan, int32_t nparts, double tflops, double gbs, double lat_us,
                          double* t1);

/* ---- diagnostics (no reference counterpart; tools/determinism*.py) ----------------------
 * Reads of a one-GPU handle's factorization, for reproducibility checks: per supernode s a hash
 * of its factor values (L panel + U12 bit patterns) and one of its row permutation,
 * out[2s], out[2s+1] (2 * nsuper entries); its values as stored (L panel M x ns, ld M, then U12
 * ns x nu, ld ns); its offsets (Loff, Uoff, Foff (-1: no F22), M; 4 * nsuper entries); and
 * doubles [off, off+cnt) of the factor store (which 0) or the front scratch (which 1) -- cnt < 0
 * returns the buffer's length in *len.  Each synchronises the handle's stream first. */
int smlu_dev_front_hash(smlu_handle* h, unsigned long long* out);
int smlu_dev_front_values(smlu_handle* h, int64_t s, double* out);
int smlu_dev_front_offsets(smlu_handle* h, int64_t* out);
int smlu_dev_copy(smlu_handle* h, int which, int64_t off, int64_t cnt, double* out, int64_t* len);

/* ---- environment knobs (read by the library in one place, csrc/tune.cpp; nothing else in the
 * environment changes its numerics or schedule) ---------------------------------------------
 *   SMLU_OB=w          outer block width of the blocked fronts (multiple of 64; default 384)
 *   SMLU_T128MIN=t     128x128 MFMA tiles for GEMM launches with >= t output tiles (default 512)
 *   SMLU_SMALLK=0      no one-shot k <= 64 GEMM tile (tests: forces the 64x64 VALU tile, and the
 *                      GEMM-form TRSM onto the 128 tile when SMLU_T128MIN allows it)
 *   SMLU_FULLPIV_NS=k  largest front with full-candidate pivoting (tests; default: 512, or 0
 *                      for diagonally dominant values)
 *   SMLU_SWEEP_SPIN=s  polls before a sync-free solve wait gives up and the solve is re-run on the
 *                      per-block schedule (default 2^22; 0 = at once, tests)
 *   SMLU_SOLVE_STEPS=1 per-block solve launches instead of the sync-free sweeps
 *   SMLU_NO_GRAPH      eager launches instead of captured hipGraphs
 *   SMLU_DEBUG_SYNC    synchronise after every launch (localises a failing kernel)
 *   SMLU_NO_REPIVOT    no re-pivoting refactor after weak diagonal-tile pivots (tests)
 * and, not a library knob: OMP_NUM_THREADS, when set, caps the host threads of the analysis
 * (otherwise the hardware threads, at most 32; the plan does not depend on the thread count).
 */

/* Library version string. */
const char* smlu_version(void);

#if defined(__GNUC__)
#pragma GCC visibility pop
#endif
#ifdef __cplusplus
}
#endif

#endif /* SMLU_H */
