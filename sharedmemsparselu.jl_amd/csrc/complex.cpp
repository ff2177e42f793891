// complex.cpp — ComplexF64 handles as the real-equivalent 2n x 2n operator.
#include "handle.hpp"

// ---- ComplexF64 (the reference is generic in Tf, src/SharedMemSparseLU.jl:43,64,286)
// A complex A is factored as its real-equivalent K (2n x 2n): the entry a_ij = x + iy becomes the
// 2x2 block [[x, -y], [y, x]] at rows 2i, 2i+1 and columns 2j, 2j+1.  K = L U with threshold
// pivoting is an LU of the complex operator, so every kernel of the real path (MFMA Schur
// updates included) runs unchanged, and an interleaved complex vector (re, im, re, im, ...) IS a
// vector of K: the solve entry points take complex buffers as 2n doubles.  Column 2j of K holds
// complex column j's values verbatim, column 2j+1 the pairs (-y, x).  The column order is
// computed on the complex pattern and expanded to (2k, 2k+1) pairs, so each 2x2 block stays
// inside one front.  Cost: 2x the flops and factor bytes of a native complex LU.
namespace {
struct ZExpand {
  std::vector<int64_t> colptr, rowval;   // K's pattern, in the caller's index base
  std::vector<int64_t> dst;
  std::vector<int32_t> off;
  std::vector<int64_t> zcolptr, zrowval; // the complex pattern, 0-based
  std::vector<int64_t> preorder;         // K column order (pairs)
};

std::string z_expand(int64_t n, const int64_t* colptr, const int64_t* rowval, int base, const smlu_opts& o,
                     ZExpand& Z) {
  if (n <= 0 || n >= (int64_t)INT32_MAX / 2) return "invalid n for a complex matrix";
  if (colptr[0] != base) return "colptr[0] must equal index_base";
  const int64_t nnz = colptr[n] - base;
  if (nnz < 0 || nnz > (int64_t)INT32_MAX) return "invalid nnz";
  Z.zcolptr.resize(n + 1);
  Z.zrowval.resize(nnz);
  std::vector<int32_t> r32(nnz);
  for (int64_t j = 0; j <= n; ++j) {
    Z.zcolptr[j] = colptr[j] - base;
    if (j > 0 && Z.zcolptr[j] < Z.zcolptr[j - 1]) return "colptr not monotone";
  }
  if (Z.zcolptr[n] != nnz) return "colptr not monotone";
  for (int64_t e = 0; e < nnz; ++e) {
    const int64_t r = rowval[e] - base;
    if (r < 0 || r >= n) return "row index out of range";
    Z.zrowval[e] = r;
    r32[e] = (int32_t)r;
  }
  Z.colptr.assign(2 * n + 1, base);
  Z.rowval.resize(4 * nnz);
  Z.dst.resize(nnz);
  Z.off.resize(nnz);
  for (int64_t j = 0; j < n; ++j) {
    const int64_t c0 = Z.zcolptr[j], c = Z.zcolptr[j + 1] - c0, k0 = 4 * c0;
    Z.colptr[2 * j + 1] = base + k0 + 2 * c;
    Z.colptr[2 * j + 2] = base + k0 + 4 * c;
    for (int64_t t = 0; t < c; ++t) {
      const int64_t r = Z.zrowval[c0 + t];
      Z.rowval[k0 + 2 * t] = Z.rowval[k0 + 2 * c + 2 * t] = base + 2 * r;
      Z.rowval[k0 + 2 * t + 1] = Z.rowval[k0 + 2 * c + 2 * t + 1] = base + 2 * r + 1;
      Z.dst[c0 + t] = k0 + 2 * t;
      Z.off[c0 + t] = (int32_t)(2 * c);
    }
  }
  std::string err;
  std::vector<int64_t> ord;
  if (o.ordering == SMLU_ORDER_GIVEN) return "complex handles compute their own order";
  ord = compute_order(n, Z.zcolptr.data(), r32.data(), plan_opts(o), err);
  if (!err.empty()) return err;
  if ((int64_t)ord.size() != n) return "ordering is not a permutation";
  Z.preorder.resize(2 * n);
  for (int64_t k = 0; k < n; ++k) {
    Z.preorder[2 * k] = 2 * ord[k];
    Z.preorder[2 * k + 1] = 2 * ord[k] + 1;
  }
  return "";
}

void z_values(const std::vector<int64_t>& dst, const std::vector<int32_t>& off, const double* z, double* K) {
  const int64_t nnz = (int64_t)dst.size();
  for (int64_t e = 0; e < nnz; ++e) {
    const double x = z[2 * e], y = z[2 * e + 1];
    const int64_t d = dst[e];
    K[d] = x;
    K[d + 1] = y;
    K[d + off[e]] = -y;
    K[d + off[e] + 1] = x;
  }
}

void z_adopt(smlu_handle* h, int64_t n, ZExpand& Z) {
  h->zc = true;
  h->zn = n;
  h->znnz = (int64_t)Z.dst.size();
  h->zdst.swap(Z.dst);
  h->zoff.swap(Z.off);
  h->zcolptr.swap(Z.zcolptr);
  h->zrowval.swap(Z.zrowval);
  h->d_zdst.free();
  h->d_zoff.free();
}
}  // namespace


int smlu_create_z(int64_t n, const int64_t* colptr, const int64_t* rowval, const double* nzval,
                  const smlu_opts* opts, smlu_handle** out) {
  if (!out) return fail(nullptr, SMLU_ERR_ARG, "out is NULL");
  *out = nullptr;
  if (n <= 0 || !colptr || !nzval) return fail(nullptr, SMLU_ERR_ARG, "invalid matrix arguments");
  smlu_opts o;
  if (opts) o = *opts;
  else smlu_default_opts(&o);
  if (!valid_opts(&o)) return fail(nullptr, SMLU_ERR_ARG, "index_base must be 0 or 1");
  if (colptr[n] - o.index_base > 0 && !rowval) return fail(nullptr, SMLU_ERR_ARG, "invalid matrix arguments");
  ZExpand Z;
  std::vector<double> K;
  try {
    std::string e = z_expand(n, colptr, rowval, o.index_base, o, Z);
    if (!e.empty()) return fail(nullptr, SMLU_ERR_ARG, e);
    K.resize(Z.rowval.size());
    z_values(Z.dst, Z.off, nzval, K.data());
  } catch (const std::bad_alloc&) {
    return fail(nullptr, SMLU_ERR_ALLOC, "host allocation failed");
  }
  if (o.chunk_size > 0) o.chunk_size = std::min<int64_t>(2 * o.chunk_size, 2 * n);
  int rc = create_impl(2 * n, Z.colptr.data(), Z.rowval.data(), K.data(), nullptr, nullptr, nullptr, &o, out,
                       0, 1, nullptr, nullptr, &Z.preorder);
  if (*out) z_adopt(*out, n, Z);
  return rc;
}

int smlu_refactor_z(smlu_handle* h, const double* nzval) {
  if (!h || !nzval) return fail(h, SMLU_ERR_ARG, "NULL argument");
  if (!h->zc) return fail(h, SMLU_ERR_ARG, "not a complex handle (smlu_create_z)");
  std::vector<double> K(h->plan.nnzA);
  z_values(h->zdst, h->zoff, nzval, K.data());
  return smlu_refactor(h, K.data());
}

int smlu_refactor_z_device(smlu_handle* h, const double* d_nzval) {
  if (!h || !d_nzval) return fail(h, SMLU_ERR_ARG, "NULL argument");
  if (!h->zc) return fail(h, SMLU_ERR_ARG, "not a complex handle (smlu_create_z)");
  if (reinterpret_cast<uintptr_t>(d_nzval) % 16) return fail(h, SMLU_ERR_ARG, "complex values must be 16-byte aligned");
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(after_caller(h));
  if (!h->d_zdst.p) {
    HIPCHK(h->d_zdst.upload(h->zdst.data(), h->zdst.size(), h->stream));
    HIPCHK(h->d_zoff.upload(h->zoff.data(), h->zoff.size(), h->stream));
  }
  HIPCHK(launch_expand_z(h->stream, h->znnz, d_nzval, h->d_zdst.p, h->d_zoff.p, h->A.p));
  return refactor_resident(h);
}

int smlu_refactor_csc_z(smlu_handle* h, int64_t n, const int64_t* colptr, const int64_t* rowval,
                        const double* nzval) {
  if (!h || !colptr || !rowval || !nzval) return fail(h, SMLU_ERR_ARG, "NULL argument");
  if (!h->zc) return fail(h, SMLU_ERR_ARG, "not a complex handle (smlu_create_z)");
  const int base = h->opts.index_base;
  bool same = (n == h->zn) && colptr[n] - base == h->znnz;
  for (int64_t j = 0; same && j <= n; ++j) same = (colptr[j] - base == h->zcolptr[j]);
  for (int64_t e = 0; same && e < h->znnz; ++e) same = (rowval[e] - base == h->zrowval[e]);
  if (same) return smlu_refactor_z(h, nzval);
  ZExpand Z;
  std::vector<double> K;
  try {
    std::string e = z_expand(n, colptr, rowval, base, h->opts, Z);
    if (!e.empty()) return fail(h, SMLU_ERR_ARG, e);
    K.resize(Z.rowval.size());
    z_values(Z.dst, Z.off, nzval, K.data());
  } catch (const std::bad_alloc&) {
    return fail(h, SMLU_ERR_ALLOC, "host allocation failed");
  }
  const std::vector<int64_t> pre = Z.preorder;
  z_adopt(h, n, Z);
  return refactor_csc_impl(h, 2 * n, Z.colptr.data(), Z.rowval.data(), K.data(), &pre);
}


// ---- ComplexF64 factors (F.L::SparseMatrixCSC{ComplexF64}, src/SharedMemSparseLU.jl:47-48) ----
// The handle holds the LU of K = phi(A) (phi: x + iy -> [[x, -y], [y, x]]).  When the row pivots
// kept every complex row pair together and in order (pK[2k] = 2i, pK[2k+1] = 2i + 1: always under
// diagonal pivoting, and whenever a complex pivot's real part carries its column), K's factors fold
// exactly into the complex LU B = L U of B = (Rs .* A)[p, q]:  phi(L) = L_K D^{-1} and
// phi(U) = D U_K with D = blockdiag([[1, 0], [Im u_kk / Re u_kk, 1]]), which gives
//   l_ik = L_K[2i+1, 2k+1] - i L_K[2i, 2k+1]   and   u_kj = U_K[2k, 2j] - i U_K[2k, 2j+1]
// (odd columns of L_K, even rows of U_K).  A pivot sequence that split a pair has no complex LU
// form: SMLU_ERR_STATE, and the real-equivalent factors stay available (smlu_get_factors).
struct ExportedZ {
  std::vector<int64_t> Lp, Li, Up, Ui, p, q;
  std::vector<double> Lx, Ux;   // interleaved (re, im)
};

static int export_complex(smlu_handle* h, ExportedZ& Z, bool values) {
  if (!h->zc) return fail(h, SMLU_ERR_ARG, "not a complex handle (smlu_create_z)");
  Exported X;
  int rc = export_factors(h, X, values);
  if (rc != SMLU_OK) return rc;
  const int64_t n = h->zn;
  Z.p.resize(n);
  Z.q.resize(n);
  // A pair kept in reverse order (rows 2i+1, 2i: the pair rule swapped inside the pair) is the
  // real equivalent of the complex row times -i with its second row negated (N): with
  // K_rot = N P K Q, the factors of K_rot are N L N and N U, which fold as usual to complex
  // L_c U_c = (D Rs.*A)[p, q], D = diag(-i on swapped rows); then (Rs.*A)[p, q] = L' U' with
  // L' = D^-1 L_c D (still unit lower) and U' = D^-1 U_c.
  std::vector<char> sw(n, 0);
  for (int64_t k = 0; k < n; ++k) {
    const int64_t a = X.p[2 * k], b = X.p[2 * k + 1];
    if (std::min(a, b) % 2 != 0 || std::max(a, b) != std::min(a, b) + 1)
      return fail(h, SMLU_ERR_STATE, "complex factors: the row pivots split complex row pair " + std::to_string(k) +
                                         " (only the real-equivalent factors exist; smlu_get_factors)");
    if (X.q[2 * k] % 2 != 0 || X.q[2 * k + 1] != X.q[2 * k] + 1)
      return fail(h, SMLU_ERR_STATE, "internal: complex column pair split");
    sw[k] = a > b;
    Z.p[k] = std::min(a, b) / 2;
    Z.q[k] = X.q[2 * k] / 2;
  }
  auto nsign = [&](int64_t r) { return ((r & 1) && sw[r / 2]) ? -1.0 : 1.0; };   // N's entry of K row r
  // L: complex column k from K's column 2k+1 (rows >= 2k+1); pairs (2i, 2i+1) are adjacent
  Z.Lp.assign(n + 1, 0);
  Z.Li.clear();
  Z.Lx.clear();
  for (int64_t k = 0; k < n; ++k) {
    const int64_t c = 2 * k + 1;
    for (int64_t e = X.Lp[c]; e < X.Lp[c + 1]; ++e) {
      const int64_t r = X.Li[e], i = r / 2;
      if (Z.Li.size() == (size_t)Z.Lp[k] || Z.Li.back() != i) {
        Z.Li.push_back(i);
        Z.Lx.push_back(0.0);
        Z.Lx.push_back(0.0);
      }
      const double v = values ? X.Lx[e] * nsign(r) * nsign(c) : 0.0;
      if (r & 1) Z.Lx[Z.Lx.size() - 2] = v;    // real part: row 2i+1 of the odd column
      else Z.Lx[Z.Lx.size() - 1] = -v;         // imaginary part: minus row 2i
    }
    Z.Lp[k + 1] = (int64_t)Z.Li.size();
  }
  // D^-1 L_c D: entry (i, k) times d_k / d_i, d = -i on swapped rows (x i: (re, im) -> (-im, re))
  if (values)
    for (int64_t k = 0; k < n; ++k)
      for (int64_t e = Z.Lp[k]; e < Z.Lp[k + 1]; ++e) {
        const int64_t i = Z.Li[e];
        if (sw[i] == sw[k]) continue;
        double& re = Z.Lx[2 * e];
        double& im = Z.Lx[2 * e + 1];
        const double r0 = re, i0 = im;
        if (sw[k]) { re = i0; im = -r0; }     // d_k / d_i = -i
        else { re = -i0; im = r0; }           // d_k / d_i = i
      }
  // U: complex column j from the even rows of K's columns 2j (real part) and 2j+1 (minus imaginary)
  Z.Up.assign(n + 1, 0);
  Z.Ui.clear();
  Z.Ux.clear();
  for (int64_t j = 0; j < n; ++j) {
    int64_t a = X.Up[2 * j], ae = X.Up[2 * j + 1], b = X.Up[2 * j + 1], be = X.Up[2 * j + 2];
    while (true) {
      while (a < ae && (X.Ui[a] & 1)) ++a;
      while (b < be && (X.Ui[b] & 1)) ++b;
      if (a >= ae && b >= be) break;
      const int64_t ra = a < ae ? X.Ui[a] : INT64_MAX, rb = b < be ? X.Ui[b] : INT64_MAX;
      const int64_t r = std::min(ra, rb);
      Z.Ui.push_back(r / 2);
      Z.Ux.push_back(ra == r && values ? X.Ux[a] : 0.0);
      Z.Ux.push_back(rb == r && values ? -X.Ux[b] : 0.0);
      if (ra == r) ++a;
      if (rb == r) ++b;
    }
    Z.Up[j + 1] = (int64_t)Z.Ui.size();
  }
  // D^-1 U_c: row i times 1/d_i = i on swapped rows (U's even rows are not touched by N)
  if (values)
    for (size_t e = 0; e < Z.Ui.size(); ++e)
      if (sw[Z.Ui[e]]) {
        const double r0 = Z.Ux[2 * e], i0 = Z.Ux[2 * e + 1];
        Z.Ux[2 * e] = -i0;
        Z.Ux[2 * e + 1] = r0;
      }
  return SMLU_OK;
}

int smlu_get_sizes_z(smlu_handle* h, int64_t* n, int64_t* nnzL, int64_t* nnzU) {
  if (!h) return fail(h, SMLU_ERR_ARG, "NULL handle");
  ExportedZ Z;
  int rc = export_complex(h, Z, false);
  if (rc != SMLU_OK) return rc;
  if (n) *n = h->zn;
  if (nnzL) *nnzL = Z.Lp[h->zn];
  if (nnzU) *nnzU = Z.Up[h->zn];
  return SMLU_OK;
}

int smlu_get_factors_z(smlu_handle* h, int64_t* Lcolptr, int64_t* Lrowval, double* Lnzval, int64_t* Ucolptr,
                       int64_t* Urowval, double* Unzval, int64_t* p, int64_t* q, double* Rs) {
  if (!h) return fail(h, SMLU_ERR_ARG, "NULL handle");
  if (!h->have_numeric) return fail(h, SMLU_ERR_STATE, "no numeric factorization");
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(hipStreamSynchronize(h->stream));
  ExportedZ Z;
  int rc = export_complex(h, Z, true);
  if (rc != SMLU_OK) return rc;
  const int64_t n = h->zn, b = h->opts.index_base;
  if (Lcolptr) for (int64_t j = 0; j <= n; ++j) Lcolptr[j] = Z.Lp[j] + b;
  if (Lrowval) for (size_t e = 0; e < Z.Li.size(); ++e) Lrowval[e] = Z.Li[e] + b;
  if (Lnzval) std::memcpy(Lnzval, Z.Lx.data(), sizeof(double) * Z.Lx.size());
  if (Ucolptr) for (int64_t j = 0; j <= n; ++j) Ucolptr[j] = Z.Up[j] + b;
  if (Urowval) for (size_t e = 0; e < Z.Ui.size(); ++e) Urowval[e] = Z.Ui[e] + b;
  if (Unzval) std::memcpy(Unzval, Z.Ux.data(), sizeof(double) * Z.Ux.size());
  if (p) for (int64_t i = 0; i < n; ++i) p[i] = Z.p[i] + b;
  if (q) for (int64_t i = 0; i < n; ++i) q[i] = Z.q[i] + b;
  if (Rs) {   // the real-equivalent rows 2i and 2i+1 share the scale of complex row i
    std::vector<double> rk(2 * n);
    HIPCHK(hipMemcpy(rk.data(), h->Rs.p, sizeof(double) * 2 * n, hipMemcpyDeviceToHost));
    for (int64_t i = 0; i < n; ++i) Rs[i] = rk[2 * i];
  }
  return SMLU_OK;
}

