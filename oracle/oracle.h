/* oracle.h — CPU restatement of the reference path.  TEST INFRASTRUCTURE ONLY (see oracle.c). */
#ifndef SMLU_ORACLE_H
#define SMLU_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_lu {
  int64_t n, nnzL, nnzU;
  int64_t *Lp, *Li, *Up, *Ui;
  double *Lx, *Ux;
} oracle_lu;

/* All indices 0-based.  p, q: new -> old. */
int oracle_rowscale(int64_t n, const int64_t* colptr, const int64_t* rowval, const double* nzval,
                    double* Rs);
oracle_lu* oracle_lu_fixed(int64_t n, const int64_t* colptr, const int64_t* rowval,
                           const double* nzval, const double* Rs, const int64_t* p,
                           const int64_t* q, int* status);
void oracle_lu_free(oracle_lu* F);
int64_t oracle_lu_nnz(const oracle_lu* F, int which);
void oracle_lu_export(const oracle_lu* F, int64_t* Lp, int64_t* Li, double* Lx, int64_t* Up,
                      int64_t* Ui, double* Ux);
int oracle_lsolve(int64_t n, const int64_t* Lp, const int64_t* Li, const double* Lx, double* x);
int oracle_rsolve(int64_t n, const int64_t* Up, const int64_t* Ui, const double* Ux, double* x);
int oracle_ldiv(const oracle_lu* F, const double* Rs, const int64_t* p, const int64_t* q,
                const double* b, double* x);

/* mf.c: multifrontal restatement of the GPU's pivot rule (and the multi-core CPU baseline).
 * p0, q: row pre-order and column order (new -> old); the assembly tree: first[nsup+1],
 * parent[nsup] (postorder: parent > child, -1 root), update rows rowptr[nsup+1] / rows (sorted
 * global positions); mode[nsup]: 0/1 = every fully-summed row is a candidate, 2 = the 64 x 64
 * diagonal tile (NULL: 1 everywhere). */
typedef struct oracle_mf oracle_mf;
oracle_mf* oracle_mf_create(int64_t n, const int64_t* colptr, const int64_t* rowval, const int64_t* p0,
                            const int64_t* q, int64_t nsup, const int64_t* first, const int64_t* parent,
                            const int64_t* rowptr, const int64_t* rows, const int32_t* mode,
                            double diag_tol, double piv_tol, int nthreads, int* status);
int oracle_mf_factor(oracle_mf* h, const double* nzval);
/* ComplexF64 real-equivalent K: pair-preserving pivots (mf.c: factor_front). */
void oracle_mf_set_pairs(oracle_mf* h, int pairs);
void oracle_mf_result(const oracle_mf* h, int32_t* rowperm, int32_t* flags, double* Rs);
void oracle_mf_destroy(oracle_mf* h);
/* Front s after oracle_mf_factor: L panel (M x ns, ld M) then U12 (ns x nu, ld ns); returns the
 * count of doubles (out may be NULL to query it), -1 for a bad s. */
int64_t oracle_mf_front_values(const oracle_mf* h, int64_t s, double* out);
int oracle_dominant(int64_t n, const int64_t* colptr, const int64_t* rowval, const double* a);

#ifdef __cplusplus
}
#endif
#endif
