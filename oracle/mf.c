/*
 * mf.c — multifrontal CPU restatement of the numeric factorization with the pivot RULE of the
 * GPU path.  TEST INFRASTRUCTURE ONLY: only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg load it (through oracle.py); libsmlu.so never links or calls it.
 *
 * Why it exists.  The reference's pivot order comes from UMFPACK's threshold partial pivoting
 * inside lu(A) / lu!(F, A) (/root/reference/src/SharedMemSparseLU.jl:74, :247; p, q, Rs
 * extracted at :75-77, :93-94).  oracle.c factors (Rs.*A)[p, q] for a GIVEN p; this file CHOOSES
 * p independently, so the GPU's pivot decisions are checked against a restatement instead of
 * being fed back to the checker.  Given the analysis (column order q, row pre-order p0, the
 * assembly tree: supernode partition, parents, update rows of every front) it replays the
 * documented rule of the GPU kernels with plain C arithmetic:
 *
 *  - fronts are assembled from the scaled entries Rs[i]*a_ij of (Rs.*A)[p0, q] and the
 *    children's Schur complements, children in ascending (postorder) order;
 *  - each front eliminates its ns fully-summed columns with threshold partial pivoting over a
 *    candidate set of its fully-summed rows.  The diagonal test is UMFPACK's symmetric-strategy
 *    rule (its published default Control[UMFPACK_SYM_PIVOT_TOLERANCE] = 0.001, the library's
 *    default diag_tol): a_kk is kept when |a_kk| >= diag_tol * max|candidate| and a_kk != 0;
 *    otherwise the candidate of largest magnitude (smallest position on ties).  UMFPACK would
 *    instead take, among the candidates passing its 0.1 threshold, the row of least degree -- a
 *    sparsity criterion that has no meaning inside a dense front;
 *  - candidate set per front mode: 0/1 = every remaining fully-summed row, 2 = the remaining rows
 *    of the 64 x 64 diagonal tile holding the column;
 *  - flags per front: 1 = a candidate column is entirely zero (singular), 2 = a weak pivot: a
 *    multiplier of magnitude above 1/pivot_tol in a non-candidate row (mode 0: |pivot| below
 *    pivot_tol times the column maximum over all rows below), i.e. a pivot that fails UMFPACK's
 *    threshold test against the rows it could not choose from.
 * The mode of each front and the re-pivoting decision (weak/singular tile pivots -> every
 * blocked front re-factored with full candidates) are restated in oracle.py.
 *
 * The same code, with mode 1 everywhere, OpenMP over the fronts of an assembly-tree level and
 * inside the large fronts, and cache-blocked updates, is bench.py's multi-core CPU baseline: a
 * partial-pivoting multifrontal LU of one matrix on all host cores.
 */
#include "oracle.h"

#include <malloc.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

struct oracle_mf {
  int64_t n, nnz, nsup, nlev;
  int64_t *first, *parent, *rowptr, *rows;
  int32_t* mode;
  int64_t *chptr, *chlist;      /* children of each front, ascending */
  int64_t *levptr, *levlist;    /* fronts by height in the assembly tree */
  int64_t *aptr, *aent;         /* A entries per front */
  int32_t *alr, *alc;           /* their local row / column */
  int64_t *arow;                /* original row of each of those entries (Rs) */
  int32_t* relmap;              /* per update row: local index in the parent front */
  int64_t *loff, *uoff;         /* factor store: L panel (M x ns) and U12 (ns x nu) */
  double* store;
  double** f22;                 /* live contribution blocks */
  double* Rs;
  int32_t *rowperm, *flags;     /* per position: local pre-swap row; per front: flags */
  int64_t *colptr, *rowval;     /* pattern copy (row scaling) */
  double diag_tol, piv_tol;
  int nthreads;
  int pairs;                    /* ComplexF64 real-equivalent: pair-preserving pivots (below) */
  double* work;                 /* flops of each front's subtree (task cut-off) */
};

static int64_t ns_of(const oracle_mf* h, int64_t s) { return h->first[s + 1] - h->first[s]; }
static int64_t nu_of(const oracle_mf* h, int64_t s) { return h->rowptr[s + 1] - h->rowptr[s]; }

/* local index of global position g inside front s (-1 if absent) */
static int64_t local_index(const oracle_mf* h, int64_t s, int64_t g) {
  const int64_t f = h->first[s], ns = ns_of(h, s);
  if (g >= f && g < f + ns) return g - f;
  int64_t lo = h->rowptr[s], hi = h->rowptr[s + 1];
  while (lo < hi) {
    int64_t mid = (lo + hi) / 2;
    if (h->rows[mid] < g) lo = mid + 1;
    else hi = mid;
  }
  return (lo < h->rowptr[s + 1] && h->rows[lo] == g) ? ns + (lo - h->rowptr[s]) : -1;
}

void oracle_mf_destroy(oracle_mf* h) {
  if (!h) return;
  free(h->first); free(h->parent); free(h->rowptr); free(h->rows); free(h->mode);
  free(h->chptr); free(h->chlist); free(h->levptr); free(h->levlist);
  free(h->aptr); free(h->aent); free(h->alr); free(h->alc); free(h->arow);
  free(h->relmap); free(h->loff); free(h->uoff); free(h->store);
  if (h->f22)
    for (int64_t s = 0; s < h->nsup; ++s) free(h->f22[s]);
  free(h->f22); free(h->Rs); free(h->rowperm); free(h->flags);
  free(h->colptr); free(h->rowval); free(h->work);
  free(h);
}

#define ALLOC(p, cnt) do { (p) = calloc((size_t)((cnt) > 0 ? (cnt) : 1), sizeof(*(p))); if (!(p)) goto fail; } while (0)

oracle_mf* oracle_mf_create(int64_t n, const int64_t* colptr, const int64_t* rowval, const int64_t* p0,
                            const int64_t* q, int64_t nsup, const int64_t* first, const int64_t* parent,
                            const int64_t* rowptr, const int64_t* rows, const int32_t* mode,
                            double diag_tol, double piv_tol, int nthreads, int* status) {
  *status = 0;
  /* front and contribution blocks are allocated and freed per factorization: keep them on the
   * heap (no mmap/munmap and page faults per front once the heap has grown) */
  mallopt(M_MMAP_THRESHOLD, 1 << 30);
  mallopt(M_TRIM_THRESHOLD, 1 << 30);
  oracle_mf* h = calloc(1, sizeof(oracle_mf));
  int64_t *p0inv = NULL, *qinv = NULL, *col2s = NULL, *cnt = NULL, *efront = NULL;
  if (!h) { *status = -3; return NULL; }
  const int64_t nnz = colptr[n];
  h->n = n; h->nnz = nnz; h->nsup = nsup;
  h->diag_tol = diag_tol; h->piv_tol = piv_tol;
  h->nthreads = nthreads > 0 ? nthreads : 1;
  ALLOC(h->first, nsup + 1); ALLOC(h->parent, nsup); ALLOC(h->rowptr, nsup + 1);
  ALLOC(h->rows, rowptr[nsup]); ALLOC(h->mode, nsup);
  memcpy(h->first, first, (nsup + 1) * sizeof(int64_t));
  memcpy(h->parent, parent, nsup * sizeof(int64_t));
  memcpy(h->rowptr, rowptr, (nsup + 1) * sizeof(int64_t));
  if (rowptr[nsup] > 0) memcpy(h->rows, rows, rowptr[nsup] * sizeof(int64_t));
  for (int64_t s = 0; s < nsup; ++s) h->mode[s] = mode ? mode[s] : 1;
  ALLOC(h->colptr, n + 1); ALLOC(h->rowval, nnz);
  memcpy(h->colptr, colptr, (n + 1) * sizeof(int64_t));
  if (nnz > 0) memcpy(h->rowval, rowval, nnz * sizeof(int64_t));
  /* children (ascending) and levels (height) */
  ALLOC(h->chptr, nsup + 1); ALLOC(h->chlist, nsup);
  for (int64_t s = 0; s < nsup; ++s)
    if (parent[s] >= 0) h->chptr[parent[s] + 1]++;
  for (int64_t s = 0; s < nsup; ++s) h->chptr[s + 1] += h->chptr[s];
  ALLOC(cnt, nsup + 1);
  for (int64_t s = 0; s < nsup; ++s)
    if (parent[s] >= 0) h->chlist[h->chptr[parent[s]] + cnt[parent[s]]++] = s;
  {
    int64_t* lev = cnt;   /* reuse: height of each front (children have smaller indices) */
    int64_t mx = 0;
    for (int64_t s = 0; s < nsup; ++s) {
      int64_t l = 0;
      for (int64_t c = h->chptr[s]; c < h->chptr[s + 1]; ++c)
        if (lev[h->chlist[c]] + 1 > l) l = lev[h->chlist[c]] + 1;
      lev[s] = l;
      if (l > mx) mx = l;
      if (parent[s] >= 0 && parent[s] <= s) { *status = -1; goto fail; }   /* postorder required */
    }
    h->nlev = mx + 1;
    ALLOC(h->levptr, h->nlev + 1); ALLOC(h->levlist, nsup);
    for (int64_t s = 0; s < nsup; ++s) h->levptr[lev[s] + 1]++;
    for (int64_t l = 0; l < h->nlev; ++l) h->levptr[l + 1] += h->levptr[l];
    int64_t* pos = malloc((h->nlev + 1) * sizeof(int64_t));
    if (!pos) goto fail;
    memcpy(pos, h->levptr, (h->nlev + 1) * sizeof(int64_t));
    for (int64_t s = 0; s < nsup; ++s) h->levlist[pos[lev[s]]++] = s;
    free(pos);
  }
  /* relmap */
  ALLOC(h->relmap, rowptr[nsup]);
  for (int64_t s = 0; s < nsup; ++s)
    for (int64_t e = rowptr[s]; e < rowptr[s + 1]; ++e) {
      if (parent[s] < 0) { *status = -1; goto fail; }
      int64_t li = local_index(h, parent[s], rows[e]);
      if (li < 0) { *status = -1; goto fail; }
      h->relmap[e] = (int32_t)li;
    }
  /* A entries -> front slots of (Rs.*A)[p0, q] */
  ALLOC(p0inv, n); ALLOC(qinv, n); ALLOC(col2s, n);
  for (int64_t k = 0; k < n; ++k) { p0inv[p0[k]] = k; qinv[q[k]] = k; }
  for (int64_t s = 0; s < nsup; ++s)
    for (int64_t k = first[s]; k < first[s + 1]; ++k) col2s[k] = s;
  ALLOC(h->aptr, nsup + 1); ALLOC(h->aent, nnz); ALLOC(h->alr, nnz); ALLOC(h->alc, nnz); ALLOC(h->arow, nnz);
  ALLOC(efront, nnz);
  for (int64_t j = 0; j < n; ++j)
    for (int64_t e = colptr[j]; e < colptr[j + 1]; ++e) {
      const int64_t r = p0inv[rowval[e]], c = qinv[j];
      const int64_t s = col2s[r < c ? r : c];   /* L part: column c's front; U part: row r's front */
      const int64_t lr = local_index(h, s, r), lc = local_index(h, s, c);
      if (lr < 0 || lc < 0) { *status = -1; goto fail; }
      efront[e] = s;
      h->alr[e] = (int32_t)lr;   /* by entry for now, permuted to front order below */
      h->alc[e] = (int32_t)lc;
      h->aptr[s + 1]++;
    }
  for (int64_t s = 0; s < nsup; ++s) h->aptr[s + 1] += h->aptr[s];
  memset(cnt, 0, (nsup + 1) * sizeof(int64_t));
  for (int64_t e = 0; e < nnz; ++e) h->aent[h->aptr[efront[e]] + cnt[efront[e]]++] = e;
  {
    int32_t* tr = malloc((size_t)(nnz > 0 ? nnz : 1) * sizeof(int32_t));
    int32_t* tc = malloc((size_t)(nnz > 0 ? nnz : 1) * sizeof(int32_t));
    if (!tr || !tc) { free(tr); free(tc); goto fail; }
    for (int64_t t = 0; t < nnz; ++t) {
      tr[t] = h->alr[h->aent[t]];
      tc[t] = h->alc[h->aent[t]];
      h->arow[t] = rowval[h->aent[t]];
    }
    free(h->alr); free(h->alc);
    h->alr = tr; h->alc = tc;
  }
  /* factor store */
  ALLOC(h->loff, nsup); ALLOC(h->uoff, nsup);
  {
    int64_t off = 0;
    for (int64_t s = 0; s < nsup; ++s) {
      const int64_t ns = ns_of(h, s), nu = nu_of(h, s);
      h->loff[s] = off; off += (ns + nu) * ns;
      h->uoff[s] = off; off += ns * nu;
    }
    ALLOC(h->store, off);
    /* touch every page of the factor store now (calloc hands out lazily zeroed pages), so the first
     * factorization is not charged the page faults (bench.py times it without a warm-up run) */
#pragma omp parallel for num_threads(h->nthreads) schedule(static)
    for (int64_t i = 0; i < off; i += 512) h->store[i] = 0.0;
  }
  ALLOC(h->work, nsup);
  for (int64_t s = 0; s < nsup; ++s) {   /* children precede parents */
    const double ns = (double)ns_of(h, s), M = ns + (double)nu_of(h, s);
    h->work[s] += 2.0 * M * M * ns;
    if (parent[s] >= 0) h->work[parent[s]] += h->work[s];
  }
  ALLOC(h->f22, nsup); ALLOC(h->Rs, n); ALLOC(h->rowperm, n); ALLOC(h->flags, nsup);
  free(p0inv); free(qinv); free(col2s); free(cnt); free(efront);
  return h;
fail:
  if (*status == 0) *status = -3;
  free(p0inv); free(qinv); free(col2s); free(cnt); free(efront);
  oracle_mf_destroy(h);
  return NULL;
}

typedef double v4d __attribute__((vector_size(32)));   /* AVX2 (x86-64-v3) */

static inline v4d ldu4(const double* p) {
  v4d v;
  memcpy(&v, p, sizeof v);
  return v;
}
static inline void stu4(double* p, v4d v) { memcpy(p, &v, sizeof v); }

/* 8 x 4 register block of C -= A * B over k0..k1 (A column-major: 8 contiguous rows). */
static inline void micro_8x4(int64_t kk, const double* A, int64_t lda, const double* B, int64_t ldb, double* C,
                             int64_t ldc) {
  v4d c00 = ldu4(C), c01 = ldu4(C + 4);
  v4d c10 = ldu4(C + ldc), c11 = ldu4(C + ldc + 4);
  v4d c20 = ldu4(C + 2 * ldc), c21 = ldu4(C + 2 * ldc + 4);
  v4d c30 = ldu4(C + 3 * ldc), c31 = ldu4(C + 3 * ldc + 4);
  for (int64_t k = 0; k < kk; ++k) {
    const v4d a0 = ldu4(A + k * lda), a1 = ldu4(A + k * lda + 4);
    const double* b = B + k;
    const v4d b0 = {b[0], b[0], b[0], b[0]};
    const v4d b1 = {b[ldb], b[ldb], b[ldb], b[ldb]};
    const v4d b2 = {b[2 * ldb], b[2 * ldb], b[2 * ldb], b[2 * ldb]};
    const v4d b3 = {b[3 * ldb], b[3 * ldb], b[3 * ldb], b[3 * ldb]};
    c00 -= a0 * b0; c01 -= a1 * b0;
    c10 -= a0 * b1; c11 -= a1 * b1;
    c20 -= a0 * b2; c21 -= a1 * b2;
    c30 -= a0 * b3; c31 -= a1 * b3;
  }
  stu4(C, c00); stu4(C + 4, c01);
  stu4(C + ldc, c10); stu4(C + ldc + 4, c11);
  stu4(C + 2 * ldc, c20); stu4(C + 2 * ldc + 4, c21);
  stu4(C + 3 * ldc, c30); stu4(C + 3 * ldc + 4, c31);
}

/* C[m x n] -= A[m x k] * B[k x n], column-major: 8 x 4 register blocks (AVX2 FMA) over k blocks
 * of 256 and row blocks of 96 (the A block stays in L2, its 8-row slice in L1 across the
 * column steps); the column blocks are OpenMP tasks when par != 0. */
static void gemm_sub(int64_t m, int64_t n, int64_t k, const double* A, int64_t lda, const double* B,
                     int64_t ldb, double* C, int64_t ldc, int par) {
  if (m <= 0 || n <= 0 || k <= 0) return;
  const int64_t MB = 96, KB = 256, NB = 64;
  const int64_t nbn = (n + NB - 1) / NB;
#pragma omp taskloop grainsize(1) if (par && nbn > 1)
  for (int64_t jb = 0; jb < nbn; ++jb) {
    const int64_t j0 = jb * NB, j1 = j0 + NB < n ? j0 + NB : n;
    for (int64_t k0 = 0; k0 < k; k0 += KB) {
      const int64_t k1 = k0 + KB < k ? k0 + KB : k, kk = k1 - k0;
      for (int64_t i0 = 0; i0 < m; i0 += MB) {
        const int64_t i1 = i0 + MB < m ? i0 + MB : m;
        const int64_t i8 = i0 + ((i1 - i0) / 8) * 8;
        int64_t j = j0;
        for (; j + 4 <= j1; j += 4) {
          for (int64_t i = i0; i < i8; i += 8)
            micro_8x4(kk, A + i + k0 * lda, lda, B + k0 + j * ldb, ldb, C + i + j * ldc, ldc);
          for (int64_t jj = j; jj < j + 4; ++jj)     /* leftover rows */
            for (int64_t kq = k0; kq < k1; ++kq) {
              const double b = B[jj * ldb + kq];
              for (int64_t i = i8; i < i1; ++i) C[jj * ldc + i] -= A[kq * lda + i] * b;
            }
        }
        for (; j < j1; ++j)                           /* leftover columns */
          for (int64_t kq = k0; kq < k1; ++kq) {
            const double b = B[j * ldb + kq];
            for (int64_t i = i0; i < i1; ++i) C[j * ldc + i] -= A[kq * lda + i] * b;
          }
      }
    }
  }
}

/* Factor one assembled front W (M x M, column-major, ld M): ns pivots with the candidate rule of
 * `mode`, blocked right-looking (panels of NBP columns, trailing update by gemm_sub).
 * perm[0..ns): local pre-swap row of each position.  Returns the front's flags. */
/* Pair-preserving pivot rule of a ComplexF64 handle's real-equivalent K (rows and columns 2i, 2i+1
 * of complex row/column i stay adjacent; every front starts at an even position).  Even column k:
 * candidate pairs (e, e+1), e even, of squared magnitude x^2 + y^2 (fma(x, x, y * y), K column k
 * holds x, y of the complex entry); the diagonal pair is kept when its squared magnitude is at
 * least diag_tol^2 times the largest and nonzero, else the first largest pair; inside the chosen
 * pair the row of larger |value| in column k becomes the pivot row (a swap inside the pair is the
 * complex row times -i up to a sign, folded back at export).  Odd column k: the pair's other row,
 * no search.  The GPU kernels (kernels_front.hip, SNode.cpair) restate the same rule. */
static void swap_rows(double* W, int64_t M, int64_t a, int64_t b, int32_t* perm) {
  if (a == b) return;
  for (int64_t j = 0; j < M; ++j) {
    const double t = W[j * M + a];
    W[j * M + a] = W[j * M + b];
    W[j * M + b] = t;
  }
  const int32_t t = perm[a]; perm[a] = perm[b]; perm[b] = t;
}

static int factor_front(double* W, int64_t M, int64_t ns, int mode, double diag_tol, double piv_tol,
                        int32_t* perm, int par, int pairs) {
  const int64_t NBP = 32;
  int flags = 0;
  for (int64_t i = 0; i < ns; ++i) perm[i] = (int32_t)i;
  for (int64_t kb = 0; kb < ns; kb += NBP) {
    const int64_t ke = kb + NBP < ns ? kb + NBP : ns;
    int64_t second = -1;   /* pairs: position of the current pair's other row */
    for (int64_t k = kb; k < ke; ++k) {
      double* col = W + k * M;
      if (pairs) {
        if ((k & 1) == 0) {
          int64_t cend = ns;
          if (mode == 2) {
            const int64_t t0 = (k / 64) * 64;
            cend = t0 + 64 < ns ? t0 + 64 : ns;
          }
          double am = 0.0, amo = 0.0;
          int64_t ai = k;
          for (int64_t e = k; e < cend; e += 2) {
            const double v = fma(col[e], col[e], col[e + 1] * col[e + 1]);
            if (v > am) { am = v; ai = e; }
          }
          for (int64_t e = cend; e < M; e += 2) {
            const double v = fma(col[e], col[e], col[e + 1] * col[e + 1]);
            if (v > amo) amo = v;
          }
          const double d2 = fma(col[k], col[k], col[k + 1] * col[k + 1]);
          int64_t pc = k;
          if (am <= 0.0) flags |= 1;
          else if (!(d2 >= diag_tol * diag_tol * am && d2 != 0.0)) pc = ai;
          const int64_t r1 = fabs(col[pc + 1]) > fabs(col[pc]) ? pc + 1 : pc;
          const int64_t r2 = 2 * pc + 1 - r1;
          if (am > 0.0) {
            const double pm = fma(col[pc], col[pc], col[pc + 1] * col[pc + 1]);
            if (mode == 0) {
              if (pm < piv_tol * piv_tol * (am > amo ? am : amo)) flags |= 2;
            } else if (amo > pm / (piv_tol * piv_tol)) {
              flags |= 2;
            }
          }
          swap_rows(W, M, k, r1, perm);
          second = r2 == k ? r1 : r2;
        } else {
          swap_rows(W, M, k, second, perm);
          if (col[k] == 0.0) flags |= 1;
        }
        const double pinv = 1.0 / col[k];
        if (col[k] != 0.0)
          for (int64_t i = k + 1; i < M; ++i) col[i] *= pinv;
        for (int64_t j = k + 1; j < ke; ++j) {
          double* cj = W + j * M;
          const double u = cj[k];
          if (u != 0.0)
            for (int64_t i = k + 1; i < M; ++i) cj[i] -= col[i] * u;
        }
        continue;
      }
      int64_t cend = ns;
      if (mode == 2) {
        const int64_t t0 = (k / 64) * 64;
        cend = t0 + 64 < ns ? t0 + 64 : ns;
      }
      double am = 0.0, amo = 0.0;
      int64_t ai = k;
      for (int64_t i = k; i < cend; ++i) {
        const double v = fabs(col[i]);
        if (v > am) { am = v; ai = i; }
      }
      for (int64_t i = cend; i < M; ++i) {
        const double v = fabs(col[i]);
        if (v > amo) amo = v;
      }
      int64_t piv = k;
      if (am <= 0.0) {
        flags |= 1;
      } else if (!(fabs(col[k]) >= diag_tol * am && col[k] != 0.0)) {
        piv = ai;
      }
      if (piv != k) {   /* interchange rows k and piv across the whole front */
        for (int64_t j = 0; j < M; ++j) {
          double t = W[j * M + k];
          W[j * M + k] = W[j * M + piv];
          W[j * M + piv] = t;
        }
        int32_t t = perm[k]; perm[k] = perm[piv]; perm[piv] = t;
      }
      const double pv = col[k];
      if (am > 0.0) {
        if (mode == 0) {
          if (fabs(pv) < piv_tol * (am > amo ? am : amo)) flags |= 2;
        } else if (amo / fabs(pv) > 1.0 / piv_tol) {
          flags |= 2;
        }
      }
      const double pinv = 1.0 / pv;
      for (int64_t i = k + 1; i < M; ++i) col[i] *= pinv;
      /* update the rest of the panel (columns k+1 .. ke) */
      for (int64_t j = k + 1; j < ke; ++j) {
        double* cj = W + j * M;
        const double u = cj[k];
        if (u != 0.0)
          for (int64_t i = k + 1; i < M; ++i) cj[i] -= col[i] * u;
      }
    }
    if (ke >= M) continue;
    /* U12 rows of the panel: L11^{-1} W[kb:ke, ke:M] (unit lower), then the trailing update */
    const int64_t w = ke - kb, nr = M - ke;
#pragma omp taskloop grainsize(64) if (par && nr > 256)
    for (int64_t j = ke; j < M; ++j) {
      double* cj = W + j * M;
      for (int64_t k = kb; k < ke; ++k) {
        const double x = cj[k];
        if (x != 0.0)
          for (int64_t i = k + 1; i < ke; ++i) cj[i] -= W[k * M + i] * x;
      }
    }
    gemm_sub(nr, nr, w, W + kb * M + ke, M, W + ke * M + kb, M, W + ke * M + ke, M, par);
  }
  return flags;
}

/* Assemble, factor and store front s; its Schur complement goes to h->f22[s]. */
static int do_front(oracle_mf* h, const double* nzval, int64_t s, int par) {
  const int64_t ns = ns_of(h, s), nu = nu_of(h, s), M = ns + nu;
  double* W = calloc((size_t)(M * M), sizeof(double));
  if (!W) return -3;
  for (int64_t t = h->aptr[s]; t < h->aptr[s + 1]; ++t) {
    const int64_t e = h->aent[t];
    W[(int64_t)h->alc[t] * M + h->alr[t]] = h->Rs[h->arow[t]] * nzval[e];
  }
  for (int64_t c = h->chptr[s]; c < h->chptr[s + 1]; ++c) {
    const int64_t ch = h->chlist[c], nuc = nu_of(h, ch);
    const int32_t* rm = h->relmap + h->rowptr[ch];
    const double* F = h->f22[ch];
    for (int64_t jc = 0; jc < nuc; ++jc) {
      double* wc = W + (int64_t)rm[jc] * M;
      for (int64_t ic = 0; ic < nuc; ++ic) wc[rm[ic]] += F[jc * nuc + ic];
    }
    free(h->f22[ch]);
    h->f22[ch] = NULL;
  }
  int32_t* perm = h->rowperm + h->first[s];
  h->flags[s] = factor_front(W, M, ns, h->mode[s], h->diag_tol, h->piv_tol, perm, par, h->pairs);
  memcpy(h->store + h->loff[s], W, (size_t)(M * ns) * sizeof(double));
  for (int64_t j = 0; j < nu; ++j)
    memcpy(h->store + h->uoff[s] + j * ns, W + (ns + j) * M, (size_t)ns * sizeof(double));
  if (nu > 0) {
    double* F = malloc((size_t)(nu * nu) * sizeof(double));
    if (!F) { free(W); return -3; }
    for (int64_t j = 0; j < nu; ++j) memcpy(F + j * nu, W + (ns + j) * M + ns, (size_t)nu * sizeof(double));
    h->f22[s] = F;
  }
  free(W);
  return 0;
}

/* Front s after its children: the assembly tree as OpenMP tasks (children in parallel, the
 * front when all of them are done); fronts with enough work also split their updates into
 * tasks (taskloop over column blocks). */
static void front_task(oracle_mf* h, const double* nzval, int64_t s, int* err) {
  for (int64_t c = h->chptr[s]; c < h->chptr[s + 1]; ++c) {
    const int64_t ch = h->chlist[c];
#pragma omp task firstprivate(ch) shared(err) if (h->nthreads > 1 && h->work[ch] > 2e6)
    front_task(h, nzval, ch, err);
  }
#pragma omp taskwait
  const int64_t ns = ns_of(h, s), M = ns + nu_of(h, s);
  const int r = do_front(h, nzval, s, h->nthreads > 1 && (double)M * M * ns > 5e7);
  if (r) {
#pragma omp atomic write
    *err = 1;
  }
}

/* One numeric factorization (row scaling + every front).  Returns 0, or 1 when some front
 * flagged a zero candidate column, negative on allocation failure. */
void oracle_mf_set_pairs(oracle_mf* h, int pairs) { h->pairs = pairs; }

int oracle_mf_factor(oracle_mf* h, const double* nzval) {
  oracle_rowscale(h->n, h->colptr, h->rowval, nzval, h->Rs);
  int err = 0;
#pragma omp parallel num_threads(h->nthreads)
#pragma omp single
  {
    for (int64_t s = 0; s < h->nsup; ++s)
      if (h->parent[s] < 0) {
#pragma omp task firstprivate(s) shared(err)
        front_task(h, nzval, s, &err);
      }
#pragma omp taskwait
  }
  if (err) return -3;
  for (int64_t s = 0; s < h->nsup; ++s) {
    free(h->f22[s]);
    h->f22[s] = NULL;
  }
  for (int64_t s = 0; s < h->nsup; ++s)
    if (h->flags[s] & 1) return 1;
  return 0;
}

void oracle_mf_result(const oracle_mf* h, int32_t* rowperm, int32_t* flags, double* Rs) {
  if (rowperm) memcpy(rowperm, h->rowperm, (size_t)h->n * sizeof(int32_t));
  if (flags) memcpy(flags, h->flags, (size_t)h->nsup * sizeof(int32_t));
  if (Rs) memcpy(Rs, h->Rs, (size_t)h->n * sizeof(double));
}

/* Front s's factor values as stored after the last factorization: its L panel (M x ns, ld M: the
 * unit-lower multipliers below the diagonal, U11 on and above it, rows in pivot order) followed by
 * U12 (ns x nu, ld ns) -- the layout of the GPU's smlu_dev_front_values, so the two compare entry
 * by entry on the same assembly tree.  Returns the number of doubles written (M ns + ns nu). */
int64_t oracle_mf_front_values(const oracle_mf* h, int64_t s, double* out) {
  if (s < 0 || s >= h->nsup) return -1;
  const int64_t ns = ns_of(h, s), nu = nu_of(h, s), M = ns + nu;
  if (out) {
    memcpy(out, h->store + h->loff[s], (size_t)(M * ns) * sizeof(double));
    if (nu > 0) memcpy(out + M * ns, h->store + h->uoff[s], (size_t)(ns * nu) * sizeof(double));
  }
  return M * ns + ns * nu;
}

/* Diagonal dominance by columns or by rows (|a_jj| >= sum of the other |a_ij| with a_jj != 0),
 * sequential sums in CSC order: the test the GPU path applies to every new set of values to pick
 * its pivoting mode.  Returns 1 / 0. */
int oracle_dominant(int64_t n, const int64_t* colptr, const int64_t* rowval, const double* a) {
  double* rd = calloc((size_t)(n > 0 ? n : 1), sizeof(double));
  double* ro = calloc((size_t)(n > 0 ? n : 1), sizeof(double));
  if (!rd || !ro) { free(rd); free(ro); return -3; }
  int col_dom = 1;
  for (int64_t j = 0; j < n; ++j) {
    double d = 0.0, off = 0.0;
    for (int64_t e = colptr[j]; e < colptr[j + 1]; ++e) {
      const double v = fabs(a[e]);
      if (rowval[e] == j) { d += v; rd[j] += v; }
      else { off += v; ro[rowval[e]] += v; }
    }
    if (!(d > 0.0 && d >= off)) col_dom = 0;
  }
  int row_dom = 1;
  for (int64_t i = 0; i < n && !col_dom; ++i)
    if (!(rd[i] > 0.0 && rd[i] >= ro[i])) row_dom = 0;
  free(rd); free(ro);
  return col_dom || row_dom;
}
