/*
 * oracle.c — CPU restatement of the reference's numeric path.  TEST INFRASTRUCTURE ONLY:
 * only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this.
 * The product (libsmlu.so) never links or calls it.
 *
 * What it restates (reference = /root/reference, SharedMemSparseLU.jl @ 2024-10-20):
 *  - Row scaling Rs[i] = 1 / sum_j |a_ij| (UMFPACK default SUM scaling; the multiplicative
 *    convention of the relation F.L*F.U == (F.Rs .* A)[F.p, F.q], src/SharedMemSparseLU.jl:307).
 *    A zero row keeps Rs = 1.
 *  - The numeric factorization lu(A)/lu!(F,A) (:74, :247) for a FIXED pivot sequence (p, q):
 *    left-looking Gilbert-Peierls column elimination of B = (Rs.*A)[p,q] with no further
 *    pivoting.  L: unit lower, explicit unit diagonal stored first, rows sorted.  U: upper,
 *    rows sorted, diagonal last (UMFPACK's CSC extraction convention).
 *  - ldiv! (:286-342): wrk = Rs[p] .* b[p]; L \ wrk; U \ wrk; x[q] = wrk.
 *  - lsolve!/rsolve! semantics (:349-392) as plain CSC triangular solves (the verbatim
 *    chunked trsv/gemm restatement lives in oracle.py).
 * The third-party numerics the reference calls (SuiteSparse UMFPACK, OpenBLAS) are not
 * vendored under /root/reference and are not installed here; parity of this oracle is
 * pinned by the reference's own test checks (test/runtests.jl) restated in tests/, by the
 * UMFPACK contract above, and by LAPACK (scipy) known answers for dense LU — see DESIGN.md.
 */
#include "oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

int oracle_rowscale(int64_t n, const int64_t* colptr, const int64_t* rowval, const double* nzval,
                    double* Rs) {
  for (int64_t i = 0; i < n; ++i) Rs[i] = 0.0;
  for (int64_t j = 0; j < n; ++j)
    for (int64_t e = colptr[j]; e < colptr[j + 1]; ++e) Rs[rowval[e]] += fabs(nzval[e]);
  for (int64_t i = 0; i < n; ++i) Rs[i] = (Rs[i] > 0.0) ? 1.0 / Rs[i] : 1.0;
  return 0;
}

typedef struct {
  int64_t cap, len;
  int64_t* idx;
  double* val;
} vec_t;

static int vpush(vec_t* v, int64_t i, double x) {
  if (v->len == v->cap) {
    int64_t nc = v->cap ? 2 * v->cap : 1024;
    int64_t* ni = (int64_t*)realloc(v->idx, nc * sizeof(int64_t));
    if (!ni) return -1;
    v->idx = ni;
    double* nv = (double*)realloc(v->val, nc * sizeof(double));
    if (!nv) return -1;
    v->val = nv;
    v->cap = nc;
  }
  v->idx[v->len] = i;
  v->val[v->len] = x;
  v->len++;
  return 0;
}

static int cmp_pair(const void* a, const void* b) {
  const int64_t* x = (const int64_t*)a;
  const int64_t* y = (const int64_t*)b;
  return (x[0] > y[0]) - (x[0] < y[0]);
}

/* sort column segment [s, e) of (idx, val) by idx */
static void sort_col(int64_t* idx, double* val, int64_t s, int64_t e, int64_t* tmp) {
  int64_t m = e - s;
  if (m <= 1) return;
  for (int64_t t = 0; t < m; ++t) {
    tmp[2 * t] = idx[s + t];
    memcpy(&tmp[2 * t + 1], &val[s + t], sizeof(double));
  }
  qsort(tmp, (size_t)m, 2 * sizeof(int64_t), cmp_pair);
  for (int64_t t = 0; t < m; ++t) {
    idx[s + t] = tmp[2 * t];
    memcpy(&val[s + t], &tmp[2 * t + 1], sizeof(double));
  }
}

oracle_lu* oracle_lu_fixed(int64_t n, const int64_t* colptr, const int64_t* rowval,
                           const double* nzval, const double* Rs, const int64_t* p,
                           const int64_t* q, int* status) {
  *status = 0;
  oracle_lu* F = (oracle_lu*)calloc(1, sizeof(oracle_lu));
  int64_t* pinv = (int64_t*)malloc(n * sizeof(int64_t));
  double* x = (double*)calloc(n, sizeof(double));
  int64_t* mark = (int64_t*)malloc(n * sizeof(int64_t));
  int64_t* stack = (int64_t*)malloc(n * sizeof(int64_t));
  int64_t* pstack = (int64_t*)malloc(n * sizeof(int64_t));
  int64_t* topo = (int64_t*)malloc(n * sizeof(int64_t));
  int64_t* Lp = (int64_t*)malloc((n + 1) * sizeof(int64_t));
  int64_t* Up = (int64_t*)malloc((n + 1) * sizeof(int64_t));
  vec_t L = {0, 0, NULL, NULL}, U = {0, 0, NULL, NULL};
  if (!F || !pinv || !x || !mark || !stack || !pstack || !topo || !Lp || !Up) {
    *status = -3;
    goto fail;
  }
  for (int64_t k = 0; k < n; ++k) pinv[p[k]] = k;
  for (int64_t k = 0; k < n; ++k) mark[k] = -1;
  Lp[0] = Up[0] = 0;
  for (int64_t k = 0; k < n; ++k) {
    int64_t c = q[k];
    /* symbolic reach of B(:,k) in the graph of L(:, 0:k-1) -> topo[top..n) */
    int64_t top = n;
    for (int64_t e = colptr[c]; e < colptr[c + 1]; ++e) {
      int64_t i = pinv[rowval[e]];
      if (mark[i] == k) continue;
      /* iterative DFS from i */
      int64_t head = 0;
      stack[0] = i;
      while (head >= 0) {
        int64_t j = stack[head];
        if (mark[j] != k) {
          mark[j] = k;
          pstack[head] = (j < k) ? Lp[j] + 1 : 0; /* skip unit diagonal (stored first) */
        }
        int done = 1;
        if (j < k) {
          int64_t end = Lp[j + 1];
          for (int64_t t = pstack[head]; t < end; ++t) {
            int64_t r = L.idx[t];
            if (mark[r] == k) continue;
            pstack[head] = t + 1;
            stack[++head] = r;
            done = 0;
            break;
          }
        }
        if (done) {
          --head;
          topo[--top] = j;
        }
      }
    }
    /* numeric: scatter B(:,k) then eliminate in topological order */
    for (int64_t e = colptr[c]; e < colptr[c + 1]; ++e) {
      int64_t r = rowval[e];
      x[pinv[r]] += Rs[r] * nzval[e];
    }
    for (int64_t t = top; t < n; ++t) {
      int64_t j = topo[t];
      if (j >= k) continue;
      double xj = x[j];
      for (int64_t s = Lp[j] + 1; s < Lp[j + 1]; ++s) x[L.idx[s]] -= L.val[s] * xj;
    }
    double piv = x[k];
    if (piv == 0.0 || !isfinite(piv)) {
      if (*status == 0) *status = 1;
    }
    /* U(:,k): rows j <= k (diagonal last after sorting); L(:,k): unit diag then rows > k */
    int64_t ustart = U.len, lstart = L.len;
    if (vpush(&L, k, 1.0)) { *status = -3; goto fail; }
    for (int64_t t = top; t < n; ++t) {
      int64_t j = topo[t];
      if (j <= k) {
        if (vpush(&U, j, x[j])) { *status = -3; goto fail; }
      } else {
        if (vpush(&L, j, x[j] / piv)) { *status = -3; goto fail; }
      }
      x[j] = 0.0;
    }
    /* the diagonal may be structurally absent from B(:,k) and the reach: still store it */
    if (mark[k] != k) {
      if (vpush(&U, k, 0.0)) { *status = -3; goto fail; }
      if (*status == 0) *status = 1;
    }
    Up[k + 1] = U.len;
    Lp[k + 1] = L.len;
    (void)ustart;
    (void)lstart;
  }
  /* sort rows within columns */
  {
    int64_t mx = 0;
    for (int64_t k = 0; k < n; ++k) {
      if (Lp[k + 1] - Lp[k] > mx) mx = Lp[k + 1] - Lp[k];
      if (Up[k + 1] - Up[k] > mx) mx = Up[k + 1] - Up[k];
    }
    int64_t* tmp = (int64_t*)malloc((2 * mx + 2) * sizeof(int64_t));
    if (!tmp) { *status = -3; goto fail; }
    for (int64_t k = 0; k < n; ++k) {
      sort_col(L.idx, L.val, Lp[k], Lp[k + 1], tmp);
      sort_col(U.idx, U.val, Up[k], Up[k + 1], tmp);
    }
    free(tmp);
  }
  F->n = n;
  F->nnzL = L.len;
  F->nnzU = U.len;
  F->Lp = Lp;
  F->Li = L.idx;
  F->Lx = L.val;
  F->Up = Up;
  F->Ui = U.idx;
  F->Ux = U.val;
  free(pinv);
  free(x);
  free(mark);
  free(stack);
  free(pstack);
  free(topo);
  return F;
fail:
  free(pinv);
  free(x);
  free(mark);
  free(stack);
  free(pstack);
  free(topo);
  free(Lp);
  free(Up);
  free(L.idx);
  free(L.val);
  free(U.idx);
  free(U.val);
  free(F);
  return NULL;
}

void oracle_lu_free(oracle_lu* F) {
  if (!F) return;
  free(F->Lp);
  free(F->Li);
  free(F->Lx);
  free(F->Up);
  free(F->Ui);
  free(F->Ux);
  free(F);
}

int64_t oracle_lu_nnz(const oracle_lu* F, int which) { return which == 0 ? F->nnzL : F->nnzU; }

void oracle_lu_export(const oracle_lu* F, int64_t* Lp, int64_t* Li, double* Lx, int64_t* Up,
                      int64_t* Ui, double* Ux) {
  if (Lp) memcpy(Lp, F->Lp, (F->n + 1) * sizeof(int64_t));
  if (Li) memcpy(Li, F->Li, F->nnzL * sizeof(int64_t));
  if (Lx) memcpy(Lx, F->Lx, F->nnzL * sizeof(double));
  if (Up) memcpy(Up, F->Up, (F->n + 1) * sizeof(int64_t));
  if (Ui) memcpy(Ui, F->Ui, F->nnzU * sizeof(int64_t));
  if (Ux) memcpy(Ux, F->Ux, F->nnzU * sizeof(double));
}

/* L \ x in place (unit diagonal stored first in each column). */
int oracle_lsolve(int64_t n, const int64_t* Lp, const int64_t* Li, const double* Lx, double* x) {
  for (int64_t j = 0; j < n; ++j) {
    double xj = x[j];
    for (int64_t s = Lp[j]; s < Lp[j + 1]; ++s)
      if (Li[s] != j) x[Li[s]] -= Lx[s] * xj;
  }
  return 0;
}

/* U \ x in place (diagonal last in each column). */
int oracle_rsolve(int64_t n, const int64_t* Up, const int64_t* Ui, const double* Ux, double* x) {
  for (int64_t j = n - 1; j >= 0; --j) {
    int64_t d = Up[j + 1] - 1;
    if (d < Up[j] || Ui[d] != j) return -1;
    x[j] /= Ux[d];
    double xj = x[j];
    for (int64_t s = Up[j]; s < d; ++s) x[Ui[s]] -= Ux[s] * xj;
  }
  return 0;
}

/* ldiv!(x, F, b): src/SharedMemSparseLU.jl:318-339.  x may alias b. */
int oracle_ldiv(const oracle_lu* F, const double* Rs, const int64_t* p, const int64_t* q,
                const double* b, double* x) {
  int64_t n = F->n;
  double* wrk = (double*)malloc(n * sizeof(double));
  if (!wrk) return -3;
  for (int64_t i = 0; i < n; ++i) wrk[i] = Rs[p[i]] * b[p[i]];
  oracle_lsolve(n, F->Lp, F->Li, F->Lx, wrk);
  int rc = oracle_rsolve(n, F->Up, F->Ui, F->Ux, wrk);
  for (int64_t i = 0; i < n; ++i) x[q[i]] = wrk[i];
  free(wrk);
  return rc;
}
