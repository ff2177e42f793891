// export.cpp — F.L, F.U, F.p, F.q, F.Rs (src/SharedMemSparseLU.jl:45-52) from the device factors,
// and the UMFPACK pattern hand-over (smlu_create_with_pivots).
#include "handle.hpp"

static int export_exact(smlu_handle* h, Exported& X, const std::vector<double>* store,
                        const std::vector<int32_t>& rp) {
  const Plan& P = h->plan;
  const int64_t n = P.n;
  std::vector<int64_t> pinv(n);
  for (int64_t i = 0; i < n; ++i) pinv[X.p[i]] = i;
  std::vector<int64_t> Lp(n + 1, 0), Up(n + 1, 0), Li, Ui;
  std::vector<int64_t> mark(n, -1), stack(n), pstack(n), reach;
  reach.reserve(1024);
  for (int64_t k = 0; k < n; ++k) {
    const int64_t c = X.q[k];
    reach.clear();
    for (int64_t e = P.Acolptr[c]; e < P.Acolptr[c + 1]; ++e) {
      const int64_t i0 = pinv[P.Arow[e]];
      if (mark[i0] == k) continue;
      int64_t head = 0;
      stack[0] = i0;
      mark[i0] = k;
      pstack[0] = i0 < k ? Lp[i0] : 0;
      while (head >= 0) {
        const int64_t j = stack[head];
        bool pushed = false;
        if (j < k) {
          for (int64_t t = pstack[head]; t < Lp[j + 1]; ++t) {
            const int64_t r = Li[t];
            if (mark[r] == k) continue;
            pstack[head] = t + 1;
            mark[r] = k;
            stack[++head] = r;
            pstack[head] = r < k ? Lp[r] : 0;
            pushed = true;
            break;
          }
        }
        if (!pushed) {
          reach.push_back(j);
          --head;
        }
      }
    }
    if (mark[k] != k) reach.push_back(k);
    std::sort(reach.begin(), reach.end());
    for (int64_t j : reach) (j <= k ? Ui : Li).push_back(j);
    Lp[k + 1] = (int64_t)Li.size();   // strictly lower rows only (unit diagonal added below)
    Up[k + 1] = (int64_t)Ui.size();
  }
  auto front_row = [&](int64_t s, int64_t g) -> int64_t {   // local index of update row g in s
    const int32_t* b = P.s_rows.data() + P.s_rowptr[s];
    const int32_t* e = P.s_rows.data() + P.s_rowptr[s + 1];
    const int32_t* it = std::lower_bound(b, e, (int32_t)g);
    return (it == e || *it != g) ? -1 : P.ns(s) + (it - b);
  };
  X.Lp.assign(n + 1, 0);
  for (int64_t k = 0; k < n; ++k) X.Lp[k + 1] = X.Lp[k] + 1 + (Lp[k + 1] - Lp[k]);
  X.Li.resize(X.Lp[n]);
  X.Lx.resize(X.Lp[n]);
  for (int64_t k = 0; k < n; ++k) {
    const int64_t s = P.col2s[k], f = P.s_first[s], ns = P.ns(s), M = P.M(s), jj = k - f;
    int64_t o = X.Lp[k];
    X.Li[o] = k;
    X.Lx[o++] = 1.0;
    for (int64_t t = Lp[k]; t < Lp[k + 1]; ++t, ++o) {
      const int64_t i = Li[t];
      X.Li[o] = i;
      X.Lx[o] = 0.0;
      if (!store) continue;
      int64_t li = i - f;
      if (i >= f + ns) {
        const int64_t gpre = P.s_first[P.col2s[i]] + rp[i];   // position before the interchanges
        li = front_row(s, gpre);
        if (li < 0) return fail(h, SMLU_ERR_STATE, "internal: structural L entry outside its front");
      }
      X.Lx[o] = (*store)[P.Loff[s] + jj * M + li];
    }
  }
  X.Up = Up;
  X.Ui = Ui;
  X.Ux.assign(Ui.size(), 0.0);
  if (store)
    for (int64_t k = 0; k < n; ++k)
      for (int64_t t = Up[k]; t < Up[k + 1]; ++t) {
        const int64_t i = Ui[t];
        const int64_t s = P.col2s[i], f = P.s_first[s], ns = P.ns(s), M = P.M(s), jj = i - f;
        if (k < f + ns) {
          X.Ux[t] = (*store)[P.Loff[s] + (k - f) * M + jj];
        } else {
          const int64_t li = front_row(s, k);
          if (li < 0) return fail(h, SMLU_ERR_STATE, "internal: structural U entry outside its front");
          X.Ux[t] = (*store)[P.Uoff[s] + (li - ns) * ns + jj];
        }
      }
  return SMLU_OK;
}

int export_factors(smlu_handle* h, Exported& X, bool values) {
  const Plan& P = h->plan;
  const int64_t n = P.n;
  std::vector<double> store;
  if (values) {
    store.resize((size_t)P.factor_size);
    HIPCHK(hipMemcpy(store.data(), h->store.p, sizeof(double) * P.factor_size, hipMemcpyDeviceToHost));
  }
  std::vector<int32_t> rp(n);
  HIPCHK(hipMemcpy(rp.data(), h->rowperm.p, sizeof(int32_t) * n, hipMemcpyDeviceToHost));
  // final position of pre-swap position g: first + inv(rowperm)[g - first]
  std::vector<int64_t> fin(n);
  std::vector<char> swapped(P.nsup, 0);
  for (int64_t s = 0; s < P.nsup; ++s) {
    int64_t f = P.s_first[s];
    for (int64_t i = f; i < P.s_first[s + 1]; ++i) {
      fin[f + rp[i]] = i;
      if (rp[i] != i - f) swapped[s] = 1;
    }
  }
  X.p.resize(n);
  X.q.assign(P.q.begin(), P.q.end());
  for (int64_t s = 0; s < P.nsup; ++s) {
    int64_t f = P.s_first[s];
    for (int64_t i = f; i < P.s_first[s + 1]; ++i) X.p[i] = P.p0[f + rp[i]];
  }
  bool any_swap = false;
  for (int64_t s = 0; s < P.nsup && !any_swap; ++s) any_swap = swapped[s] != 0;
  // The fronts are built on pattern(A + A'); when that is not the structure of the factors
  // (unsymmetric A, row interchanges, a given p != q) the export takes the exact structural
  // pattern of (Rs.*A)[p, q] for the final (p, q) and reads each entry from its front.
  if (!P.sym_pattern || any_swap || X.p != X.q) return export_exact(h, X, values ? &store : nullptr, rp);
  // Row lists per column (L) in final positions with values; U by rows then transposed.
  X.Lp.assign(n + 1, 0);
  std::vector<int64_t> Ucnt(n + 1, 0);
  struct Ent { int64_t r; double v; };
  std::vector<std::vector<Ent>> Lcols(n), Urows(n);
  for (int64_t s = 0; s < P.nsup; ++s) {
    const int64_t f = P.s_first[s], ns = P.ns(s), nu = P.nu(s), M = ns + nu;
    const int32_t* R = P.s_rows.data() + P.s_rowptr[s];
    const double* Lpn = values ? store.data() + P.Loff[s] : nullptr;
    const double* U12 = values ? store.data() + P.Uoff[s] : nullptr;
    for (int64_t jj = 0; jj < ns; ++jj) {
      const int64_t j = f + jj;
      // structure of column j: exact (t-supernode) unless this front swapped rows
      int64_t last_own;
      const int32_t* Rb;
      int64_t Rn;
      if (!swapped[s]) {
        int64_t t = P.col2t[j];
        last_own = P.t_first[t + 1] - 1;
        Rb = P.t_rows.data() + P.t_rowptr[t];
        Rn = P.t_rowptr[t + 1] - P.t_rowptr[t];
      } else {
        last_own = f + ns - 1;
        Rb = R;
        Rn = nu;
      }
      auto& Lc = Lcols[j];
      Lc.reserve((size_t)(last_own - j + 1 + Rn));
      Lc.push_back({j, 1.0});
      for (int64_t i = j + 1; i <= last_own; ++i) {
        double v = values ? Lpn[jj * M + (i - f)] : 0.0;
        Lc.push_back({i, v});
      }
      // update rows: local index in front = ns + position in R_s
      int64_t k = 0;
      for (int64_t e = 0; e < Rn; ++e) {
        int64_t g = Rb[e];
        if (g <= f + ns - 1) {  // (exact structure may list rows inside the relaxed supernode)
          double v = values ? Lpn[jj * M + (g - f)] : 0.0;
          Lc.push_back({g, v});  // own positions: already final
          continue;
        }
        while (R[k] < g) ++k;
        double v = values ? Lpn[jj * M + ns + k] : 0.0;
        Lc.push_back({fin[g], v});
      }
      // U row j: diag block columns j..last_own and update columns
      auto& Ur = Urows[j];
      for (int64_t c = j; c <= last_own; ++c) {
        double v = values ? Lpn[(c - f) * M + jj] : 0.0;
        Ur.push_back({c, v});
      }
      k = 0;
      for (int64_t e = 0; e < Rn; ++e) {
        int64_t g = Rb[e];
        if (g <= f + ns - 1) {
          double v = values ? Lpn[(g - f) * M + jj] : 0.0;
          Ur.push_back({g, v});
          continue;
        }
        while (R[k] < g) ++k;
        double v = values ? U12[k * ns + jj] : 0.0;
        Ur.push_back({g, v});
      }
    }
  }
  for (int64_t j = 0; j < n; ++j) {
    auto& c = Lcols[j];
    std::sort(c.begin() + 1, c.end(), [](const Ent& a, const Ent& b) { return a.r < b.r; });
    X.Lp[j + 1] = X.Lp[j] + (int64_t)c.size();
  }
  X.Li.resize(X.Lp[n]);
  X.Lx.resize(X.Lp[n]);
  for (int64_t j = 0; j < n; ++j) {
    int64_t o = X.Lp[j];
    for (auto& e : Lcols[j]) { X.Li[o] = e.r; X.Lx[o] = e.v; ++o; }
  }
  // U: transpose rows -> CSC columns; rows within a column come out sorted (row-major sweep)
  for (int64_t i = 0; i < n; ++i)
    for (auto& e : Urows[i]) Ucnt[e.r + 1]++;
  X.Up.assign(n + 1, 0);
  for (int64_t j = 0; j < n; ++j) X.Up[j + 1] = X.Up[j] + Ucnt[j + 1];
  X.Ui.resize(X.Up[n]);
  X.Ux.resize(X.Up[n]);
  std::vector<int64_t> pos(X.Up.begin(), X.Up.end() - 1);
  for (int64_t i = 0; i < n; ++i)
    for (auto& e : Urows[i]) {
      X.Ui[pos[e.r]] = i;
      X.Ux[pos[e.r]] = e.v;
      pos[e.r]++;
    }
  return SMLU_OK;
}

// Exported factors restricted to the caller's L/U pattern (smlu_create_with_pivots with patterns):
// every given entry must be an entry of the structural fill X holds (else SMLU_ERR_PATTERN); the
// fill entries the caller's pattern leaves out are counted in h->pattern_dropped.
static int project_to_given(smlu_handle* h, Exported& X) {
  const int64_t n = h->plan.n;
  int64_t dropped = 0;
  auto one = [&](const std::vector<int64_t>& gp, const std::vector<int64_t>& gi, std::vector<int64_t>& xp,
                 std::vector<int64_t>& xi, std::vector<double>& xv, const char* which) -> int {
    std::vector<double> v(gi.size(), 0.0);
    for (int64_t j = 0; j < n; ++j) {
      int64_t t = xp[j];
      const int64_t te = xp[j + 1];
      for (int64_t e = gp[j]; e < gp[j + 1]; ++e) {
        while (t < te && xi[t] < gi[e]) ++t;
        if (t == te || xi[t] != gi[e])
          return fail(h, SMLU_ERR_PATTERN, std::string("given ") + which + " entry (" + std::to_string(gi[e]) + ", " +
                                               std::to_string(j) + ") is not in the structural fill of (Rs.*A)[p, q]");
        if (!xv.empty()) v[e] = xv[t];
        ++t;
      }
      dropped += (xp[j + 1] - xp[j]) - (gp[j + 1] - gp[j]);
    }
    xp = gp;
    xi = gi;
    if (!xv.empty()) xv.swap(v);
    return SMLU_OK;
  };
  int rc = one(h->gLp, h->gLi, X.Lp, X.Li, X.Lx, "L");
  if (rc != SMLU_OK) return rc;
  rc = one(h->gUp, h->gUi, X.Up, X.Ui, X.Ux, "U");
  if (rc != SMLU_OK) return rc;
  h->pattern_dropped = dropped;
  return SMLU_OK;
}

static int export_given(smlu_handle* h, Exported& X, bool values) {
  int rc = export_factors(h, X, values);
  if (rc != SMLU_OK || !h->given_pattern) return rc;
  return project_to_given(h, X);
}

// A caller's CSC pattern of L (unit diagonal stored first in each column) or U (diagonal last),
// rows strictly increasing, index base `base` -> 0-based arrays; "" or what is wrong.
static std::string read_factor_pattern(int64_t n, const int64_t* cp, const int64_t* ri, int64_t base, bool lower,
                                       std::vector<int64_t>& P, std::vector<int64_t>& I) {
  if (!cp || !ri) return "pattern arrays missing";
  if (cp[0] != base) return "colptr[0] must equal index_base";
  P.assign(n + 1, 0);
  for (int64_t j = 0; j <= n; ++j) P[j] = cp[j] - base;
  for (int64_t j = 0; j < n; ++j)
    if (P[j + 1] <= P[j]) return "every column must hold its diagonal entry";
  I.resize(P[n]);
  for (int64_t j = 0; j < n; ++j)
    for (int64_t e = P[j]; e < P[j + 1]; ++e) {
      const int64_t r = ri[e] - base;
      if (r < 0 || r >= n || (e > P[j] && r <= I[e - 1])) return "row indices out of range or not increasing";
      if (lower ? r < j : r > j) return lower ? "L entry above the diagonal" : "U entry below the diagonal";
      I[e] = r;
    }
  for (int64_t j = 0; j < n; ++j)
    if ((lower ? I[P[j]] : I[P[j + 1] - 1]) != j)
      return lower ? "L: unit diagonal must be stored first" : "U: diagonal must be stored last";
  return "";
}

int smlu_create_with_pivots(int64_t n, const int64_t* colptr, const int64_t* rowval,
                            const double* nzval, const int64_t* p, const int64_t* q,
                            const double* Rs, const int64_t* Lcolptr, const int64_t* Lrowval,
                            const int64_t* Ucolptr, const int64_t* Urowval, const smlu_opts* opts,
                            smlu_handle** out) {
  if (!p || !q) return fail(nullptr, SMLU_ERR_ARG, "p and q are required");
  const bool pat = Lcolptr || Lrowval || Ucolptr || Urowval;
  std::vector<int64_t> Lp, Li, Up, Ui;
  if (pat) {
    if (n <= 0) return fail(nullptr, SMLU_ERR_ARG, "invalid matrix arguments");
    const int64_t base = opts ? opts->index_base : 1;
    std::string e;
    try {
      e = read_factor_pattern(n, Lcolptr, Lrowval, base, true, Lp, Li);
      if (e.empty()) e = read_factor_pattern(n, Ucolptr, Urowval, base, false, Up, Ui);
    } catch (const std::bad_alloc&) {
      return fail(nullptr, SMLU_ERR_ALLOC, "host allocation failed");
    }
    if (!e.empty()) return fail(nullptr, SMLU_ERR_PATTERN, "given L/U pattern: " + e);
  }
  int rc = create_impl(n, colptr, rowval, nzval, p, q, Rs, opts, out);
  if (rc < 0 || !pat || !*out) return rc;
  smlu_handle* h = *out;
  // the caller's pattern against the structural fill of (Rs.*A)[p, q] of the plan
  h->gLp.swap(Lp);
  h->gLi.swap(Li);
  h->gUp.swap(Up);
  h->gUi.swap(Ui);
  h->given_pattern = true;
  Exported X;
  int r2 = export_given(h, X, false);
  if (r2 != SMLU_OK) {
    const std::string msg = h->err;
    smlu_destroy(h);
    *out = nullptr;
    return fail(nullptr, r2, msg);
  }
  return rc;
}

int smlu_get_sizes(smlu_handle* h, int64_t* n, int64_t* nnzL, int64_t* nnzU) {
  if (!h) return fail(h, SMLU_ERR_ARG, "NULL handle");
  Exported X;
  int rc = export_given(h, X, false);
  if (rc != SMLU_OK) return rc;
  if (n) *n = h->plan.n;
  if (nnzL) *nnzL = X.Lp[h->plan.n];
  if (nnzU) *nnzU = X.Up[h->plan.n];
  return SMLU_OK;
}

int smlu_get_factors(smlu_handle* h, int64_t* Lcolptr, int64_t* Lrowval, double* Lnzval,
                     int64_t* Ucolptr, int64_t* Urowval, double* Unzval, int64_t* p, int64_t* q,
                     double* Rs) {
  if (!h) return fail(h, SMLU_ERR_ARG, "NULL handle");
  if (!h->have_numeric) return fail(h, SMLU_ERR_STATE, "no numeric factorization");
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(hipStreamSynchronize(h->stream));
  Exported X;
  int rc = export_given(h, X, true);
  if (rc != SMLU_OK) return rc;
  const int64_t n = h->plan.n, b = h->opts.index_base;
  if (Lcolptr) for (int64_t j = 0; j <= n; ++j) Lcolptr[j] = X.Lp[j] + b;
  if (Lrowval) for (size_t e = 0; e < X.Li.size(); ++e) Lrowval[e] = X.Li[e] + b;
  if (Lnzval) std::memcpy(Lnzval, X.Lx.data(), sizeof(double) * X.Lx.size());
  if (Ucolptr) for (int64_t j = 0; j <= n; ++j) Ucolptr[j] = X.Up[j] + b;
  if (Urowval) for (size_t e = 0; e < X.Ui.size(); ++e) Urowval[e] = X.Ui[e] + b;
  if (Unzval) std::memcpy(Unzval, X.Ux.data(), sizeof(double) * X.Ux.size());
  if (p) for (int64_t i = 0; i < n; ++i) p[i] = X.p[i] + b;
  if (q) for (int64_t i = 0; i < n; ++i) q[i] = X.q[i] + b;
  if (Rs) HIPCHK(hipMemcpy(Rs, h->Rs.p, sizeof(double) * n, hipMemcpyDeviceToHost));
  return SMLU_OK;
}

