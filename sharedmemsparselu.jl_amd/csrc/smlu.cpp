// smlu.cpp — C-ABI of libsmlu.so (include/smlu.h): handle creation and lifetime, statistics,
// the host plan API.  The other entry points live in the units listed in handle.hpp.
//
// Reference surface (SharedMemSparseLU.jl, src/SharedMemSparseLU.jl):
//   ParallelSparseLU(A, chunk_size)  :64-98   -> smlu_create
//   lu!(F, A)                        :245-279 -> smlu_refactor / smlu_refactor_csc
//   ldiv!(x, F, b)                   :286-342 -> smlu_solve
//   lsolve!(F, x) / rsolve!(F, x)    :349-392 -> smlu_lsolve / smlu_rsolve
//   F.L, F.U, F.p, F.q, F.Rs         :45-52   -> smlu_get_factors
//   cleanup_ParallelSparseLU!        :31      -> smlu_destroy
#include "handle.hpp"

namespace smlu {
thread_local std::string g_last_error;
}

static int check_device(smlu_handle* h) {
  int cnt = 0;
  hipError_t e = hipGetDeviceCount(&cnt);
  if (e != hipSuccess || cnt <= 0)
    return fail(h, SMLU_ERR_NODEVICE, "no HIP device visible (libsmlu has no CPU fallback)");
  if (h->opts.device < 0 || h->opts.device >= cnt)
    return fail(h, SMLU_ERR_NODEVICE, "opts.device out of range");
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, h->opts.device) != hipSuccess)
    return fail(h, SMLU_ERR_NODEVICE, "hipGetDeviceProperties failed");
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(h, SMLU_ERR_NODEVICE, std::string("device is ") + prop.gcnArchName + ", libsmlu is built for gfx950 only");
  h->device = h->opts.device;
  return SMLU_OK;
}

std::vector<int64_t> diagonal_match(int64_t n, const int64_t* colptr, const int64_t* rowval,
                                    const double* a, int64_t base) {
  bool need = false;
  for (int64_t j = 0; j < n && !need; ++j) {
    bool has = false;
    for (int64_t e = colptr[j] - base; e < colptr[j + 1] - base; ++e)
      if (rowval[e] - base == j) has = a[e] != 0.0;
    need = !has;
  }
  if (!need) return {};
  const int64_t nnz = colptr[n] - base;
  std::vector<int64_t> cp(n + 1);
  std::vector<int32_t> ri((size_t)std::max<int64_t>(nnz, 1));
  for (int64_t j = 0; j <= n; ++j) cp[j] = colptr[j] - base;
  for (int64_t e = 0; e < nnz; ++e) ri[e] = (int32_t)(rowval[e] - base);
  std::vector<int64_t> m = zero_free_diagonal(n, cp.data(), ri.data(), a);
  bool ident = true;
  for (int64_t j = 0; j < (int64_t)m.size() && ident; ++j) ident = m[j] == j;
  if (ident) m.clear();
  return m;
}

int create_impl(int64_t n, const int64_t* colptr, const int64_t* rowval, const double* nzval,
                const int64_t* p, const int64_t* q, const double* Rs, const smlu_opts* opts,
                smlu_handle** out, int rank, int nranks, const smlu_transport* tr, RcclState* rccl,
                const std::vector<int64_t>* preorder) {
  std::unique_ptr<RcclState> rccl_own(rccl);   // owned by the handle once it exists
  if (!out) return fail(nullptr, SMLU_ERR_ARG, "out is NULL");
  *out = nullptr;
  if (n <= 0 || !colptr || (!rowval && n > 0) || !nzval)
    return fail(nullptr, SMLU_ERR_ARG, "invalid matrix arguments");
  std::unique_ptr<smlu_handle> h(new (std::nothrow) smlu_handle());
  if (!h) return fail(nullptr, SMLU_ERR_ALLOC, "allocation failed");
  h->rccl = rccl_own.release();
  if (tr) h->tr = *tr;
  if (opts) h->opts = *opts;
  else smlu_default_opts(&h->opts);
  if (!valid_opts(&h->opts)) return fail(nullptr, SMLU_ERR_ARG, "index_base must be 0 or 1");
  if (h->opts.chunk_size <= 0 || h->opts.chunk_size > n) h->opts.chunk_size = std::min<int64_t>(8, n);
  int rc = check_device(h.get());
  if (rc != SMLU_OK) return rc;
  std::string e;
  try {
    std::vector<int64_t> match;
    if (!p && h->opts.ordering != SMLU_ORDER_GIVEN)
      match = diagonal_match(n, colptr, rowval, nzval, h->opts.index_base);
    PlanOptions po = plan_opts(h->opts);
    if (preorder) po.preorder = *preorder;
    e = h->plan.build(n, colptr, rowval, h->opts.index_base, po, p, q,
                      match.empty() ? nullptr : match.data());
  } catch (const std::bad_alloc&) {
    return fail(nullptr, SMLU_ERR_ALLOC, "host allocation failed during analysis");
  }
  if (!e.empty()) return fail(nullptr, SMLU_ERR_ARG, e);
  h->rank = rank;
  h->nranks = nranks;
  h->cpair = preorder != nullptr && !h->plan.matched;
  if (!p && !h->plan.matched) h->dominant = diagonally_dominant(n, colptr, rowval, nzval, h->opts.index_base);
  if (nranks > 1) {
    if (tune().ob > 0) h->ob = tune().ob;
    h->plan.compute_owners(nranks, h->ob);
    h->opts.profile = 0;   // per-kind event timing is single-GPU only
  }
  rc = setup_device(h.get());
  if (rc != SMLU_OK) { g_last_error = h->err; return rc; }
  if (h->rccl) {
    static_cast<RcclState*>(h->rccl)->stream = h->stream;
    static_cast<RcclState*>(h->rccl)->dbuf = h->d_red.p;
  }
  hipStream_t st = h->stream;
  {
    smlu_handle* hp = h.get();
    smlu_handle* h = hp;  // for HIPCHK
    HIPCHK(hipMemcpyAsync(h->A.p, nzval, sizeof(double) * h->plan.nnzA, hipMemcpyHostToDevice, st));
    if (Rs) {
      HIPCHK(hipMemcpyAsync(h->Rs.p, Rs, sizeof(double) * n, hipMemcpyHostToDevice, st));
      h->given_Rs = true;
    }
  }
  rc = run_factor(h.get());   // collective on a partitioned handle
  *out = h.release();
  return rc;
}

// =========================================================================================
// C-ABI
// =========================================================================================

void smlu_default_opts(smlu_opts* o) {
  if (!o) return;
  std::memset(o, 0, sizeof(*o));
  o->chunk_size = 8;
  o->index_base = 1;
  o->ordering = SMLU_ORDER_AUTO;
  o->scale = 1;
  o->relax = 1;
  o->pivot_tol = 0.1;
  o->diag_pivot_tol = 0.001;   // UMFPACK's symmetric-strategy default (SYM_PIVOT_TOLERANCE)
  o->device = 0;
  o->profile = 0;
  o->leaf_size = 64;
  o->use_mfma = 1;   // fp64 MFMA tiles (use_mfma = 0: the VALU tiles, a test/comparison path)
  o->refine = -1;
  o->vendor_gemm = 0;   // reserved (the vendor GEMM comparison path was removed in round 5)
}

int smlu_create(int64_t n, const int64_t* colptr, const int64_t* rowval, const double* nzval,
                const smlu_opts* opts, smlu_handle** out) {
  return create_impl(n, colptr, rowval, nzval, nullptr, nullptr, nullptr, opts, out);
}

int smlu_create_i32(int64_t n, const int32_t* colptr, const int32_t* rowval, const double* nzval,
                    const smlu_opts* opts, smlu_handle** out) {
  if (!out || !colptr || n <= 0) return fail(nullptr, SMLU_ERR_ARG, "invalid matrix arguments");
  const int64_t base = opts ? opts->index_base : 1;
  const int64_t nnz = (int64_t)colptr[n] - base;
  if (nnz < 0 || (nnz > 0 && !rowval)) return fail(nullptr, SMLU_ERR_ARG, "invalid matrix arguments");
  std::vector<int64_t> cp(colptr, colptr + n + 1), rv(rowval, rowval + nnz);
  return smlu_create(n, cp.data(), rv.data(), nzval, opts, out);
}

void smlu_destroy(smlu_handle* h) { delete h; }

const char* smlu_last_error_string(const smlu_handle* h) {
  if (h) return h->err.c_str();
  return g_last_error.c_str();
}

int64_t smlu_last_error_col(const smlu_handle* h) {
  if (!h) return -1;
  return (h->zc && h->errcol >= 0) ? h->errcol / 2 : h->errcol;   // complex handle: column of A
}

static double plan_stat(const Plan& P, const std::string& k) {
  if (k.rfind("phase_ms", 0) == 0) {   // phase_ms0 .. phase_ms9 (Plan::phase_ms)
    const int i = std::atoi(k.c_str() + 8);
    return i >= 0 && i < 12 ? P.phase_ms[i] : std::numeric_limits<double>::quiet_NaN();
  }
  if (k == "n") return (double)P.n;
  if (k == "nnzA") return (double)P.nnzA;
  if (k == "nsuper") return (double)P.nsup;
  if (k == "ntsuper") return (double)P.ntsup;
  if (k == "nlevels") return (double)P.nlevels;
  if (k == "nnzL") return P.nnzL;
  if (k == "nnzU") return P.nnzU;
  if (k == "nnzLU") return P.nnzL + P.nnzU - (double)P.n;  // one diagonal (U's) + unit L diag stored
  if (k == "upd") return P.upd;
  if (k == "dense_flops") return P.flops;
  if (k == "stored") return P.stored;
  if (k == "front_max") return (double)P.front_max;
  if (k == "ns_max") return (double)P.ns_max;
  if (k == "nu_max") return (double)P.nu_max;
  if (k == "factor_bytes") return 8.0 * (double)P.factor_size;
  if (k == "scratch_bytes") return 8.0 * (double)P.scratch_size;
  if (k == "analysis_ms") return P.analysis_ms;
  if (k == "extadd_entries") {   // child F22 entries moved by the extend-add per factorization
    double t = 0;
    for (int64_t s = 0; s < P.nsup; ++s)
      if (P.s_parent[s] >= 0) t += (double)P.nu(s) * (double)P.nu(s);
    return t;
  }
  return std::numeric_limits<double>::quiet_NaN();
}

double smlu_stat(const smlu_handle* h, const char* key) {
  if (!h || !key) return std::numeric_limits<double>::quiet_NaN();
  std::string k(key);
  if (k == "complex") return h->zc ? 1.0 : 0.0;
  if (k == "cpair") return h->cpair ? 1.0 : 0.0;
  if (k == "launches") return (double)h->nlaunch;
  if (k == "refactor_ms_last") return h->refactor_ms;
  if (k == "solve_ms_last") return h->solve_ms;
  if (k == "growth_max") return h->growth_max;
  if (k == "weak") return (double)h->weak;
  if (k == "dominant") return h->dominant ? 1.0 : 0.0;
  if (k == "pivmode") return (double)h->pivmode;
  if (k == "matched") return h->plan.matched ? 1.0 : 0.0;
  if (k == "nranks") return (double)h->nranks;
  if (k == "owned_blocks") return (double)h->lay.blocks.size();
  if (k == "comm_steps") return (double)h->comm.size();
  if (k == "comm_calls") return (double)h->comm_calls;
  if (k == "comm_bytes_sent") return h->comm_sent;
  if (k == "comm_bytes_recv") return h->comm_recv;
  if (k == "comm_bytes_sent_refactor") return h->comm_sent_fac;
  if (k == "comm_bytes_recv_refactor") return h->comm_recv_fac;
  if (k == "rccl_nranks") return h->rccl ? (double)static_cast<const RcclState*>(h->rccl)->comm_count : 0.0;
  if (k == "store_bytes_rank") return 8.0 * (double)h->lay.store_size;
  if (k == "scratch_bytes_rank") return 8.0 * (double)h->lay.scratch_size;
  if (k == "shared_fronts") {
    double c = 0;
    for (int64_t s = 0; s < h->plan.nsup && h->nranks > 1; ++s)
      if (h->plan.dist(s) && std::binary_search(h->plan.group[s].begin(), h->plan.group[s].end(), h->rank)) ++c;
    return c;
  }
  if (k == "repivots") return (double)h->repivots;
  if (k == "mode_refactors") return (double)h->mode_refactors;
  if (k == "repivot_node") return (double)h->repivot_node;
  if (k == "repivot_info") return (double)h->repivot_info;
  if (k == "repivot_growth") return h->repivot_growth;
  if (k == "repivot_node_mode" || k == "repivot_node_ns" || k == "repivot_node_nu") {
    if (h->repivot_node < 0) return -1;
    const SNode& r = h->repivot_sn;
    return k == "repivot_node_mode" ? r.mode : k == "repivot_node_ns" ? r.ns : r.nu;
  }
  if (k == "pivot_tol") return h->opts.pivot_tol;
  if (k == "diag_pivot_tol") return h->plan.given_order ? 0.0 : h->opts.diag_pivot_tol;
  if (k == "sweep_timeouts") {   // solves re-run on the per-block schedule after a sweep wait timed out
    return (double)h->sweep_timeouts;
  }
  if (k == "sweep_status") {     // the device flag itself (cleared whenever a solve reports it)
    int32_t v = 0;
    if (h->sstatus.p && hipMemcpy(&v, h->sstatus.p, sizeof v, hipMemcpyDeviceToHost) != hipSuccess) return -1;
    return v;
  }
  if (k == "solve_sweeps") {
    int64_t c = 0;
    for (const Launch& L : h->fwd) c += L.kind == K_SWEEPF;
    for (const Launch& L : h->bwd) c += L.kind == K_SWEEPB;
    return (double)c;
  }
  if (k.rfind("launches_", 0) == 0) {   // launches per kernel variant in the factor schedule
    const std::string v = k.substr(9);
    double c = 0;
    for (const Launch& L : h->fac) {
      const bool gemm = L.kind == K_GEMM || L.kind == K_GEMMU || L.kind == K_GEMMO || L.kind == K_GEMM22;
      const bool trsm = L.kind == K_TRSML;
      const bool mfma = L.aux == 131 || L.aux == 135;
      if (v == "mfma128" && gemm && mfma) ++c;
      else if (v == "mfma128_trsm" && trsm && mfma) ++c;
      else if (v == "k64" && gemm && L.aux == 65) ++c;
      else if (v == "k64_trsm" && trsm && L.aux == 65) ++c;
      else if (v == "valu64" && gemm && L.aux == 64) ++c;
      else if (v == "mfma64" && gemm && L.aux == 66) ++c;
      else if (v == "valu64_trsm" && trsm && L.aux == 64) ++c;
      else if (v == "tri_inv" && L.kind == K_TRIINV) ++c;
      else if (v == "panel_tall" && L.kind == K_PANEL && L.nwg > 512) ++c;
    }
    return c;
  }
  if (k.rfind("fronts_mode", 0) == 0) {
    const int m = std::atoi(k.c_str() + 11);
    double c = 0;
    for (const SNode& r : h->hsn) c += r.mode == m ? 1 : 0;
    return c;
  }
  if (k == "pattern_dropped") return (double)h->pattern_dropped;
  if (k == "given_pattern") return h->given_pattern ? 1.0 : 0.0;
  if (k == "status_copy_retries") return (double)h->status_copy_retries;
  if (k == "bad_info_count") return (double)h->bad_info_count;
  if (k == "bad_info_node") return (double)h->bad_info_node;
  if (k == "bad_info_word") return (double)h->bad_info_word;
  if (k == "refine_steps") return (double)h->refine_steps;
  if (k == "refine_residual") return h->refine_resid;
  if (k == "refine_berr") return h->refine_berr;
  if (k == "gemm_flops") return h->gemm_flops;
  if (k == "gemm22_flops") return h->gemm22_flops;
  if (k == "gemm_launches") return (double)h->gemm_launches;
  if (k == "gemm_bytes") return h->gemm_bytes;
  if (k == "gemm128_launches") return (double)h->gemm128_launches;
  if (k == "vendor_calls") return 0.0;   // no vendor GEMM path (round 5)
  if (k.rfind("ms_", 0) == 0) {
    std::string name = k.substr(3);
    double t = 0;
    bool found = false;
    for (int i = 0; i < K_NKIND; ++i)
      if (name == kKindName[i]) { t += h->kind_ms[i]; found = true; }
    return found ? t : std::numeric_limits<double>::quiet_NaN();
  }
  return plan_stat(h->plan, k);
}

int smlu_plan_create(int64_t n, const int64_t* colptr, const int64_t* rowval, const smlu_opts* opts,
                     smlu_plan** out) {
  if (!out || !colptr || n <= 0) return fail(nullptr, SMLU_ERR_ARG, "invalid arguments");
  smlu_opts o;
  if (opts) o = *opts;
  else smlu_default_opts(&o);
  if (!valid_opts(&o)) return fail(nullptr, SMLU_ERR_ARG, "index_base must be 0 or 1");
  std::unique_ptr<smlu_plan> p(new smlu_plan());
  std::string e = p->plan.build(n, colptr, rowval, o.index_base, plan_opts(o));
  if (!e.empty()) return fail(nullptr, SMLU_ERR_ARG, e);
  *out = p.release();
  return SMLU_OK;
}

double smlu_plan_stat(const smlu_plan* plan, const char* key) {
  if (!plan || !key) return std::numeric_limits<double>::quiet_NaN();
  return plan_stat(plan->plan, key);
}

int smlu_plan_pattern(const smlu_plan* pl, int64_t* q, int64_t* Lcolptr, int64_t* Lrowval) {
  if (!pl) return SMLU_ERR_ARG;
  const Plan& P = pl->plan;
  if (q) for (int64_t i = 0; i < P.n; ++i) q[i] = P.q[i];
  if (Lcolptr || Lrowval) {
    int64_t o = 0;
    if (Lcolptr) Lcolptr[0] = 0;
    for (int64_t j = 0; j < P.n; ++j) {
      int64_t t = P.col2t[j], last = P.t_first[t + 1] - 1;
      if (Lrowval) {
        for (int64_t i = j; i <= last; ++i) Lrowval[o++] = i;
        for (int64_t e = P.t_rowptr[t]; e < P.t_rowptr[t + 1]; ++e) Lrowval[o++] = P.t_rows[e];
      } else {
        o += last - j + 1 + P.t_rowptr[t + 1] - P.t_rowptr[t];
      }
      if (Lcolptr) Lcolptr[j + 1] = o;
    }
  }
  return SMLU_OK;
}

int smlu_plan_supernodes(const smlu_plan* pl, int64_t* first, int64_t* parent, int64_t* level) {
  if (!pl) return SMLU_ERR_ARG;
  const Plan& P = pl->plan;
  for (int64_t s = 0; s <= P.nsup; ++s)
    if (first) first[s] = P.s_first[s];
  for (int64_t s = 0; s < P.nsup; ++s) {
    if (parent) parent[s] = P.s_parent[s];
    if (level) level[s] = P.s_level[s];
  }
  return SMLU_OK;
}

static void fronts_of(const Plan& P, int64_t* first, int64_t* parent, int64_t* rowptr, int64_t* rows,
                      int64_t* p0) {
  for (int64_t s = 0; s <= P.nsup; ++s) {
    if (first) first[s] = P.s_first[s];
    if (rowptr) rowptr[s] = P.s_rowptr[s];
  }
  for (int64_t s = 0; s < P.nsup; ++s)
    if (parent) parent[s] = P.s_parent[s];
  if (rows)
    for (int64_t e = 0; e < P.s_rowptr[P.nsup]; ++e) rows[e] = P.s_rows[e];
  if (p0)
    for (int64_t i = 0; i < P.n; ++i) p0[i] = P.p0[i];
}

int smlu_plan_fronts(const smlu_plan* pl, int64_t* rowptr, int64_t* rows, int64_t* p0) {
  if (!pl) return SMLU_ERR_ARG;
  fronts_of(pl->plan, nullptr, nullptr, rowptr, rows, p0);
  return SMLU_OK;
}

int smlu_get_fronts(smlu_handle* h, int64_t* first, int64_t* parent, int64_t* rowptr, int64_t* rows,
                    int64_t* p0, int32_t* mode) {
  if (!h) return fail(h, SMLU_ERR_ARG, "NULL handle");
  fronts_of(h->plan, first, parent, rowptr, rows, p0);
  if (mode)
    for (int64_t s = 0; s < h->plan.nsup; ++s) mode[s] = h->hsn[s].mode;
  return SMLU_OK;
}

void smlu_plan_destroy(smlu_plan* p) { delete p; }

const char* smlu_version(void) { return "smlu 0.1.0 (gfx950, fp64, multifrontal)"; }


