// solve.cpp — ldiv! / lsolve! / rsolve! (src/SharedMemSparseLU.jl:286-392) on the GPU: the level
// schedule of solve launches, iterative refinement, batched right-hand sides and the chunked layout.
#include "handle.hpp"

// One solve launch for rh.n right-hand sides (x columns at w + r*rh.ldx, front vectors at
// v + r*rh.ldv); the multi-GPU kinds (K_BWDU12C, K_VCOPY) are single-vector only.
static hipError_t run_solve_launch(smlu_handle* h, const Launch& L, double* w, double* v, Rhs rh, hipStream_t st) {
  switch (L.kind) {
    case K_FWD:
      return launch_fwd(st, (int)L.cnt, h->ilist.p + L.off, h->sn.p, h->chlist.p, h->relmap.p,
                        h->rowperm.p, h->store.p, w, v, rh);
    case K_BWD:
      return launch_bwd(st, (int)L.cnt, h->ilist.p + L.off, h->sn.p, h->rows.p, h->store.p, w, v, rh);
    case K_FWDT:
      return launch_fwd_tiny(st, (int)L.cnt, h->ilist.p + L.off, h->sn.p, h->chlist.p, h->relmap.p, h->rowperm.p,
                             h->store.p, w, v, rh, (int)L.aux);
    case K_BWDT:
      return launch_bwd_tiny(st, (int)L.cnt, h->ilist.p + L.off, h->sn.p, h->rows.p, h->store.p, w, v, rh, (int)L.aux);
    case K_FWDP:
      return launch_fwd_pull(st, L.nwg, h->ftiles.p + L.off, (int)L.cnt, h->sn.p, h->rowperm.p, h->gptr.p, h->gent.p,
                             w, v, rh);
    case K_FWDG:
      return launch_fwd_gather(st, (int)L.cnt, h->ilist.p + L.off, h->sn.p, h->chlist.p, h->relmap.p,
                               h->rowperm.p, w, v, rh);
    case K_TRIF:
      return launch_tri_block(st, false, L.nwg, h->ftiles.p + L.off, (int)L.cnt, L.step, h->sn.p,
                              h->store.p, w, v, rh);
    case K_TRIB:
      return launch_tri_block(st, true, L.nwg, h->ftiles.p + L.off, (int)L.cnt, L.step, h->sn.p,
                              h->store.p, w, v, rh);
    case K_BWDU:
      return launch_bwd_u12(st, L.nwg, h->ftiles.p + L.off, (int)L.cnt, h->sn.p, h->rows.p, h->store.p, w, v,
                            rh);
    case K_SWEEPF:
    case K_SWEEPB:
      return launch_tri_sweep(st, L.kind == K_SWEEPB, L.nwg, h->ftiles.p + L.off, (int)L.cnt, h->stick.p + L.aux2,
                              h->ssync.p + L.aux, h->sxh.p + L.aux * 64 * kMultiRhs, h->sstatus.p, h->sn.p, h->store.p,
                              w, v, rh, h->sweep_spin);
    case K_BWDU12C:
      return launch_bwd_u12_cols(st, h->sn.p, L.node, h->hsn[L.node].ns, L.aux, L.aux2, (int)L.cnt, h->rows.p,
                                 h->store.p, w, h->vbuf.p);
    case K_VCOPY:
      return launch_vcopy(st, h->sn.p, L.node, h->hsn[L.node].ns, w, h->vbuf.p);
  }
  return hipErrorInvalidValue;
}

static int run_solve_dev(smlu_handle* h, const double* db, double* dx, int mode, int nrhs = 1, int64_t ldb = 0,
                         int64_t ldx = 0) {
  // mode 0: ldiv (b -> x); 1: lsolve in place on dx (final order); 2: rsolve in place.
  // nrhs > 1 (mode 0, one GPU): columns of db / dx with leading dimensions ldb / ldx.
  Plan& P = h->plan;
  if (h->nranks > 1 && mode != 0) return fail(h, SMLU_ERR_STATE, "lsolve!/rsolve! are single-GPU only");
  if (nrhs > 1 && (mode != 0 || h->nranks > 1 || nrhs > kMultiRhs))
    return fail(h, SMLU_ERR_STATE, "batched right-hand sides: ldiv on one GPU only");
  hipStream_t st = h->stream;
  auto t0 = std::chrono::steady_clock::now();
  Timer tm(h);
  hipEvent_t stop;
  HIPCHK(tm.begin(K_FWD, &stop, h->stream));
  double* w = h->wrk.p;
  double* v = h->vbuf.p;
  Rhs rh{1, (int64_t)P.n, (int64_t)h->vbuf.n};
  if (nrhs > 1) {
    if (!h->vbufm.p) HIPCHK(h->vbufm.alloc(h->vbuf.n * kMultiRhs));
    if (!h->wrkm.p) HIPCHK(h->wrkm.alloc((size_t)P.n * kMultiRhs));
    w = h->wrkm.p;
    v = h->vbufm.p;
    rh.n = nrhs;
  }
  // batches of up to SMLU_SWEEP_MAX_RHS (<= 8) right-hand sides run the sweeps (NR-wide hand-off
  // slots), wider ones the per-block launches (fwdm / bwdm)
  // batches of up to 8 run the sweeps too (round 6: the NR substitution chains interleaved,
  // tri64_rows); wider ones the per-block schedule
  constexpr int sweep_max_rhs = 8;
  const bool steps = rh.n > std::min(8, std::max(1, sweep_max_rhs)) && h->nranks == 1;
  // The sync-free sweeps' waits are bounded: a wait that gives up raises sstatus, which is read back
  // after every solve that ran them; the solve is then re-run on the per-block schedule (fwdm / bwdm,
  // bitwise the same arithmetic), so a timed-out sweep never returns a wrong x.  Partitioned handles
  // agree on the re-run (allreduce of the flag: the per-block sequences hold the same comm steps).
  const bool check = !steps && (h->ssync_n > 0 || h->nranks > 1);
  const double* src = mode == 0 ? db : dx;
  const int64_t lds = mode == 0 && ldb > 0 ? ldb : P.n;
  auto load_input = [&](const double* in, int64_t ld) -> hipError_t {
    if (mode == 0) return launch_perm_in(st, P.n, h->p0.p, h->Rs.p, in, w, nrhs, ld, rh.ldx);
    if (mode == 1) return launch_unswap(st, P.n, h->posfirst.p, h->rowperm.p, in, w);
    return hipMemcpyAsync(w, in, sizeof(double) * P.n, hipMemcpyDeviceToDevice, st);
  };
  const double* rerun_src = src;
  int64_t rerun_ld = lds;
  if (check && (mode != 0 || db == dx)) {   // the final step overwrites the input: keep a copy for a re-run
    if (!h->bstash.p) HIPCHK(h->bstash.alloc((size_t)P.n * kMultiRhs));
    HIPCHK(hipMemcpy2DAsync(h->bstash.p, sizeof(double) * P.n, src, sizeof(double) * lds, sizeof(double) * P.n,
                            (size_t)nrhs, hipMemcpyDeviceToDevice, st));
    rerun_src = h->bstash.p;
    rerun_ld = P.n;
  }
  HIPCHK(load_input(src, lds));
  // launches between communication steps (one GPU: a single segment each)
  // overlap: a level's small fronts on the side stream next to its large fronts' per-block chain
  // (batched right-hand sides: 8 per 128^3 solve 59.5 -> 57.4 ms).  Not next to the sync-free
  // sweeps, whose waiting workgroups lose CUs to them (1 rhs: 13.8 -> 15.2 ms, round 6).
  auto run_seq = [&](const std::vector<Launch>& seq, const std::vector<size_t>& seg, const std::vector<int>& cm,
                     bool overlap) {
    for (size_t k = 0; k < seg.size(); ++k) {
      if (k > 0) {
        int rc = exec_comm(h, cm[k - 1]);
        if (rc != SMLU_OK) return rc;
      }
      const size_t hi = k + 1 < seg.size() ? seg[k + 1] : seq.size();
      // a level's side launches (grp > 0, side) on the side stream: forked after everything
      // before the level, joined before the next level
      bool forked = false;
      for (size_t i = seg[k]; i < hi; ++i) {
        const Launch& L = seq[i];
        const bool first = overlap && L.grp > 0 && (i == seg[k] || seq[i - 1].grp != L.grp);
        const bool last = overlap && L.grp > 0 && (i + 1 == hi || seq[i + 1].grp != L.grp);
        if (first) {
          HIPCHK(hipEventRecord(h->fork_ev, st));
          HIPCHK(hipStreamWaitEvent(h->side, h->fork_ev, 0));
          forked = true;
        }
        HIPCHK(run_solve_launch(h, L, w, v, rh, L.side && forked ? h->side : st));
        if (last && forked) {
          HIPCHK(hipEventRecord(h->join_ev, h->side));
          HIPCHK(hipStreamWaitEvent(st, h->join_ev, 0));
          forked = false;
        }
      }
    }
    return (int)SMLU_OK;
  };
  auto sweeps = [&](bool steps) {   // steps: the per-block sequences instead of the sweeps
    if (mode != 2) {
      int rc = steps ? run_seq(h->fwdm, h->fwdm_seg, h->fwd_comm, true) : run_seq(h->fwd, h->fwd_seg, h->fwd_comm, false);
      if (rc != SMLU_OK) return rc;
    }
    if (mode != 1) {
      int rc = steps ? run_seq(h->bwdm, h->bwdm_seg, h->bwd_comm, true) : run_seq(h->bwd, h->bwd_seg, h->bwd_comm, false);
      if (rc != SMLU_OK) return rc;
    }
    return (int)SMLU_OK;
  };
  auto finish = [&]() -> hipError_t {
    if (mode == 0) return launch_perm_out(st, P.n, h->q.p, w, dx, nrhs, rh.ldx, ldx > 0 ? ldx : P.n);
    return hipMemcpyAsync(dx, w, sizeof(double) * P.n, hipMemcpyDeviceToDevice, st);
  };
  // One GPU: the forward and backward sweeps (~1,400 launches at 128^3, fixed pointers: the
  // handle's wrk / vbuf) are captured once per (mode, rhs count) into a hipGraph and replayed;
  // only the permutation kernels see the caller's b and x.
  const bool nograph = tune().no_graph;
  if (h->nranks == 1 && !nograph && !h->graph_failed) {
    const int key = mode * 256 + rh.n;
    hipGraphExec_t ex = nullptr;
    for (auto& g : h->sol_execs)
      if (g.first == key) ex = g.second;
    if (!ex) {
      hipGraph_t g = nullptr;
      HIPCHK(hipStreamBeginCapture(st, hipStreamCaptureModeRelaxed));
      int rc = sweeps(steps);
      hipError_t ec = hipStreamEndCapture(st, &g);
      if (rc == SMLU_OK && ec == hipSuccess && g) ec = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
      if (g) (void)hipGraphDestroy(g);
      if (rc != SMLU_OK || ec != hipSuccess || !ex) {
        (void)hipGetLastError();
        h->graph_failed = true;
        ex = nullptr;
      } else {
        h->sol_execs.push_back({key, ex});
      }
    }
    if (ex) HIPCHK(hipGraphLaunch(ex, st));
    else {
      int rc = sweeps(steps);
      if (rc != SMLU_OK) return rc;
    }
  } else {
    int rc = sweeps(steps);
    if (rc != SMLU_OK) return rc;
  }
  HIPCHK(finish());
  HIPCHK(tm.end(stop));
  HIPCHK(hipStreamSynchronize(st));
  tm.collect();
  if (check) {
    long long rec[16];
    int rs = read_status(h, nullptr, 0, h->sstatus.p, 1, rec);
    if (rs != SMLU_OK) return rs;
    double bad = (rec[6] & 0xffffffffll) != 0 ? 1.0 : 0.0;
    if (h->nranks > 1 && h->tr.allreduce_max(h->tr.ctx, &bad, 1) != 0)
      return fail(h, SMLU_ERR_HIP, "transport allreduce failed (sweep status)");
    if (bad != 0) {
      ++h->sweep_timeouts;
      HIPCHK(hipMemsetAsync(h->sstatus.p, 0, sizeof(int32_t), st));
      HIPCHK(load_input(rerun_src, rerun_ld));
      int rc = sweeps(true);
      if (rc != SMLU_OK) return rc;
      HIPCHK(finish());
      HIPCHK(hipStreamSynchronize(st));
    }
  }
  h->solve_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return SMLU_OK;
}


// ldiv! plus iterative refinement on the original (unscaled) A: x <- x + A \ (b - A x).  The
// diagonal-tile pivoting of large fronts cannot always keep growth below 1/pivot_tol; when a
// refactor flags such weak pivots (h->weak), refine = -1 applies up to 3 steps (the pivot-
// failure fallback).  So it does for non-dominant values factored under a diagonal
// tolerance below the pivot tolerance (UMFPACK's symmetric default 0.001 < 0.1): a diagonal kept
// at 0.001 of its column lets the factors grow up to 1000x per step, and UMFPACK's own solve
// refines by default (IRSTEP 2) for the same reason.  Stopping rule of LAPACK's dgerfs with a
// rounding floor: a correction is solved only while the componentwise backward error
// max |r|/(|A||x|+|b|) exceeds 4 unit roundoffs (2^-51; dgerfs uses 1, which a residual summed in
// fp64 rarely reaches, so it spends two extra solves to gain nothing) and at most halves the
// previous one -- an accurate solve costs one residual and no extra solve.
// Residual buffers and the column of every A entry (allocated on first use).
int ensure_residual(smlu_handle* h) {
  Plan& P = h->plan;
  const int64_t n = P.n;
  hipStream_t st = h->stream;
  if (!h->ref_b.p) {
    HIPCHK(h->ref_b.alloc((size_t)n));
    HIPCHK(h->ref_r.alloc((size_t)n));
    HIPCHK(h->ref_d.alloc((size_t)n));
    HIPCHK(h->ref_nrm.alloc(2));
  }
  if (!h->Acol.p) {
    std::vector<int32_t> ac((size_t)std::max<int64_t>(P.nnzA, 1));
    for (int64_t c = 0; c < n; ++c)
      for (int64_t e = P.Acolptr[c]; e < P.Acolptr[c + 1]; ++e) ac[e] = (int32_t)c;
    HIPCHK(h->Acol.upload(ac.data(), ac.size(), st));
  }
  return SMLU_OK;
}

static int auto_refine_steps(const smlu_handle* h) {
  if (h->opts.refine >= 0) return h->opts.refine;
  const bool diag_pref = !h->plan.given_order && !h->dominant && h->opts.diag_pivot_tol < h->opts.pivot_tol;
  return (h->weak > 0 || diag_pref) ? 3 : 0;
}

static int solve_refined(smlu_handle* h, const double* db, double* dx) {
  const int steps = auto_refine_steps(h);
  h->refine_steps = 0;
  h->refine_resid = -1;
  h->refine_berr = -1;
  if (steps == 0) return run_solve_dev(h, db, dx, 0);
  Plan& P = h->plan;
  const int64_t n = P.n;
  hipStream_t st = h->stream;
  int rc0 = ensure_residual(h);
  if (rc0 != SMLU_OK) return rc0;
  HIPCHK(hipMemcpyAsync(h->ref_b.p, db, sizeof(double) * n, hipMemcpyDeviceToDevice, st));   // db may alias dx
  int rc = run_solve_dev(h, h->ref_b.p, dx, 0);
  if (rc != SMLU_OK) return rc;
  const double ms = h->solve_ms;
  const double eps = std::ldexp(1.0, -51);   // 4 unit roundoffs
  double prev = HUGE_VAL;
  for (int it = 0; it < steps; ++it) {
    HIPCHK(hipMemsetAsync(h->ref_nrm.p, 0, 2 * sizeof(double), st));
    HIPCHK(launch_residual(st, n, h->Arowptr.p, h->Arow_ent.p, h->Acol.p, h->A.p, dx, h->ref_b.p, h->ref_r.p,
                           h->ref_nrm.p));
    long long rec[16];
    rc = read_status(h, nullptr, 0, reinterpret_cast<const int32_t*>(h->ref_nrm.p), 4, rec);
    if (rc != SMLU_OK) return rc;
    double nrm, berr;
    std::memcpy(&nrm, &rec[6], sizeof nrm);
    std::memcpy(&berr, &rec[7], sizeof berr);
    h->refine_resid = nrm;
    h->refine_berr = berr;
    if (berr <= eps || berr > 0.5 * prev) break;
    prev = berr;
    rc = run_solve_dev(h, h->ref_r.p, h->ref_d.p, 0);
    if (rc != SMLU_OK) return rc;
    HIPCHK(launch_axpy1(st, n, h->ref_d.p, dx));
    ++h->refine_steps;
  }
  HIPCHK(hipStreamSynchronize(st));
  h->solve_ms = ms;   // the plain solve's time (refinement steps reported separately)
  return SMLU_OK;
}

int smlu_residual_device(smlu_handle* h, const double* d_x, const double* d_b, double* d_r, double* nrm) {
  if (!h || !d_x || !d_b || !d_r) return fail(h, SMLU_ERR_ARG, "NULL argument");
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(after_caller(h));
  int rc = ensure_residual(h);
  if (rc != SMLU_OK) return rc;
  hipStream_t st = h->stream;
  HIPCHK(hipMemsetAsync(h->ref_nrm.p, 0, 2 * sizeof(double), st));
  HIPCHK(launch_residual(st, h->plan.n, h->Arowptr.p, h->Arow_ent.p, h->Acol.p, h->A.p, d_x, d_b, d_r,
                         h->ref_nrm.p));
  long long rec[16];
  rc = read_status(h, nullptr, 0, reinterpret_cast<const int32_t*>(h->ref_nrm.p), 2, rec);
  if (rc != SMLU_OK) return rc;
  double v;
  std::memcpy(&v, &rec[6], sizeof v);
  if (nrm) *nrm = v;
  return SMLU_OK;
}

int smlu_solve_device(smlu_handle* h, const double* d_b, double* d_x) {
  if (!h || !d_b || !d_x) return fail(h, SMLU_ERR_ARG, "NULL argument");
  if (!h->have_numeric) return fail(h, SMLU_ERR_STATE, "no numeric factorization");
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(after_caller(h));
  return solve_refined(h, d_b, d_x);
}

int smlu_solve(smlu_handle* h, const double* b, double* x) {
  if (!h || !b || !x) return fail(h, SMLU_ERR_ARG, "NULL argument");
  if (!h->have_numeric) return fail(h, SMLU_ERR_STATE, "no numeric factorization");
  HIPCHK(hipSetDevice(h->device));
  int64_t n = h->plan.n;
  HIPCHK(hipMemcpyAsync(h->wrk2.p, b, sizeof(double) * n, hipMemcpyHostToDevice, h->stream));
  int rc = solve_refined(h, h->wrk2.p, h->wrk2.p);
  if (rc != SMLU_OK) return rc;
  HIPCHK(hipMemcpyAsync(x, h->wrk2.p, sizeof(double) * n, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  return SMLU_OK;
}

// Multiple right-hand sides.  One GPU without refinement: batches of up to kMultiRhs columns go
// through the solve kernels together (each factor value read once per batch, not per column);
// otherwise (refinement, several GPUs) one refined solve per column.  d_B may alias d_X when
// ldb == ldx (the batch is permuted into the work buffer before x is written).
static int solve_multi_dev(smlu_handle* h, int64_t nrhs, const double* d_B, int64_t ldb, double* d_X,
                           int64_t ldx) {
  const int steps = auto_refine_steps(h);
  const bool batched = steps == 0 && h->nranks == 1 && nrhs > 1;
  if (!batched) {
    for (int64_t j = 0; j < nrhs; ++j) {
      int rc = solve_refined(h, d_B + j * ldb, d_X + j * ldx);
      if (rc != SMLU_OK) return rc;
    }
    return SMLU_OK;
  }
  h->refine_steps = 0;
  h->refine_resid = -1;
  double ms = 0;
  for (int64_t j = 0; j < nrhs; j += kMultiRhs) {
    const int nb = (int)std::min<int64_t>(kMultiRhs, nrhs - j);
    int rc = run_solve_dev(h, d_B + j * ldb, d_X + j * ldx, 0, nb, ldb, ldx);
    if (rc != SMLU_OK) return rc;
    ms += h->solve_ms;
  }
  h->solve_ms = ms;
  return SMLU_OK;
}

int smlu_solve_multi_device(smlu_handle* h, int64_t nrhs, const double* d_B, int64_t ldb, double* d_X,
                            int64_t ldx) {
  if (!h || nrhs < 0 || (nrhs > 0 && (!d_B || !d_X))) return fail(h, SMLU_ERR_ARG, "invalid arguments");
  if (!h->have_numeric) return fail(h, SMLU_ERR_STATE, "no numeric factorization");
  const int64_t n = h->plan.n;
  if (ldb < n || ldx < n) return fail(h, SMLU_ERR_ARG, "leading dimension smaller than n");
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(after_caller(h));
  return solve_multi_dev(h, nrhs, d_B, ldb, d_X, ldx);
}

int smlu_solve_multi(smlu_handle* h, int64_t nrhs, const double* B, int64_t ldb, double* X, int64_t ldx) {
  if (!h || nrhs < 0 || (nrhs > 0 && (!B || !X))) return fail(h, SMLU_ERR_ARG, "invalid arguments");
  if (!h->have_numeric) return fail(h, SMLU_ERR_STATE, "no numeric factorization");
  const int64_t n = h->plan.n;
  if (ldb < n || ldx < n) return fail(h, SMLU_ERR_ARG, "leading dimension smaller than n");
  HIPCHK(hipSetDevice(h->device));
  if (nrhs > 1 && h->nranks == 1 && auto_refine_steps(h) == 0) {
    if (!h->wrk2m.p) HIPCHK(h->wrk2m.alloc((size_t)n * kMultiRhs));
    double* d = h->wrk2m.p;
    for (int64_t j = 0; j < nrhs; j += kMultiRhs) {
      const int64_t nb = std::min<int64_t>(kMultiRhs, nrhs - j);
      HIPCHK(hipMemcpy2DAsync(d, sizeof(double) * n, B + j * ldb, sizeof(double) * ldb, sizeof(double) * n, nb,
                              hipMemcpyHostToDevice, h->stream));
      int rc = solve_multi_dev(h, nb, d, n, d, n);
      if (rc != SMLU_OK) return rc;
      HIPCHK(hipMemcpy2DAsync(X + j * ldx, sizeof(double) * ldx, d, sizeof(double) * n, sizeof(double) * n, nb,
                              hipMemcpyDeviceToHost, h->stream));
    }
    HIPCHK(hipStreamSynchronize(h->stream));
    return SMLU_OK;
  }
  for (int64_t j = 0; j < nrhs; ++j) {
    HIPCHK(hipMemcpyAsync(h->wrk2.p, B + j * ldb, sizeof(double) * n, hipMemcpyHostToDevice, h->stream));
    int rc = solve_refined(h, h->wrk2.p, h->wrk2.p);
    if (rc != SMLU_OK) return rc;
    HIPCHK(hipMemcpyAsync(X + j * ldx, h->wrk2.p, sizeof(double) * n, hipMemcpyDeviceToHost, h->stream));
  }
  HIPCHK(hipStreamSynchronize(h->stream));
  return SMLU_OK;
}

static int tri_solve_host(smlu_handle* h, double* x, int mode) {
  if (!h || !x) return fail(h, SMLU_ERR_ARG, "NULL argument");
  if (!h->have_numeric) return fail(h, SMLU_ERR_STATE, "no numeric factorization");
  HIPCHK(hipSetDevice(h->device));
  int64_t n = h->plan.n;
  HIPCHK(hipMemcpyAsync(h->wrk2.p, x, sizeof(double) * n, hipMemcpyHostToDevice, h->stream));
  int rc = run_solve_dev(h, nullptr, h->wrk2.p, mode);
  if (rc != SMLU_OK) return rc;
  HIPCHK(hipMemcpyAsync(x, h->wrk2.p, sizeof(double) * n, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  return SMLU_OK;
}

int smlu_lsolve(smlu_handle* h, double* x) { return tri_solve_host(h, x, 1); }
int smlu_rsolve(smlu_handle* h, double* x) { return tri_solve_host(h, x, 2); }

// ---- the reference's dense-chunk solve layout on the GPU -------------------
// Chunk geometry, negated rectangles and back-to-front U chunks exactly as
// get_chunking_parameters / allocate_chunks / fill_chunks! (src/SharedMemSparseLU.jl:101-243)
// lay them out (quirks Q1-Q4 of SURVEY appendix B), built from the current factors.
int smlu_chunked_setup(smlu_handle* h, int64_t chunk_size) {
  if (!h) return fail(h, SMLU_ERR_ARG, "NULL handle");
  if (!h->have_numeric) return fail(h, SMLU_ERR_STATE, "no numeric factorization");
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(hipStreamSynchronize(h->stream));
  Exported X;
  int rc = export_factors(h, X, true);
  if (rc != SMLU_OK) return rc;
  const int64_t n = h->plan.n, m = n;
  int64_t cs = chunk_size > 0 ? chunk_size : 8;   // :67-70
  cs = std::min(cs, n);                           // :72 (clamped with A.n)
  const int64_t T = (m + cs - 1) / cs;            // :108 (with m, quirk Q1)
  {   // the layout is dense per chunk (the reference's): refuse what cannot fit
    double total = 0;
    for (int64_t c = 0; c < T; ++c) {
      const int64_t cmin = c * cs, cmax = std::min(m, (c + 1) * cs), s = cmax - cmin;
      int64_t rmax = cmax, rmin = cmin;
      for (int64_t j = cmin; j < cmax; ++j) {
        if (X.Lp[j + 1] > X.Lp[j]) rmax = std::max(rmax, X.Li[X.Lp[j + 1] - 1] + 1);
        if (X.Up[j + 1] > X.Up[j]) rmin = std::min(rmin, X.Ui[X.Up[j]]);
      }
      total += 2.0 * s * s + (double)(rmax - cmax) * s + (double)(cmin - rmin) * s;
    }
    if (total > 4.0e9)
      return fail(h, SMLU_ERR_ALLOC, "chunked layout needs " + std::to_string(8.0 * total / 1e9) +
                                         " GB (dense chunks, as in the reference); use smlu_solve");
  }
  std::vector<ChunkDesc> desc;
  std::vector<double> data;
  // one chunk: columns [c0, c1), rectangle rows [r0, r1) (0-based)
  auto add = [&](int64_t c0, int64_t c1, int64_t r0, int64_t r1, bool upper) {
    ChunkDesc d;
    d.c0 = c0;
    d.s = c1 - c0;
    d.r0 = r0;
    d.nr = std::max<int64_t>(r1 - r0, 0);
    d.tri = (int64_t)data.size();
    data.resize(data.size() + d.s * d.s, 0.0);
    d.rect = (int64_t)data.size();
    data.resize(data.size() + d.nr * d.s, 0.0);
    const auto& Cp = upper ? X.Up : X.Lp;
    const auto& Ci = upper ? X.Ui : X.Li;
    const auto& Cx = upper ? X.Ux : X.Lx;
    for (int64_t j = c0; j < c1; ++j)
      for (int64_t e = Cp[j]; e < Cp[j + 1]; ++e) {
        const int64_t i = Ci[e];
        const bool in_tri = upper ? i >= c0 : i < c1;
        if (in_tri) data[d.tri + (j - c0) * d.s + (i - c0)] = Cx[e];
        else if (i >= r0 && i < r1) data[d.rect + (j - c0) * d.nr + (i - r0)] = -Cx[e];   // :207, :238
      }
    desc.push_back(d);
  };
  for (int64_t c = 1; c <= T; ++c) {              // L chunks, :111-123
    const int64_t cmin = (c - 1) * cs, cmax = std::min(m, c * cs);
    int64_t rmax = cmax;                          // one past the max row of the chunk's columns
    for (int64_t j = cmin; j < cmax; ++j)
      if (X.Lp[j + 1] > X.Lp[j]) rmax = std::max(rmax, X.Li[X.Lp[j + 1] - 1] + 1);
    add(cmin, cmax, cmax, rmax, false);
  }
  for (int64_t c = 1; c <= T; ++c) {              // U chunks from the back, :132-144 (Q2)
    const int64_t cmin = (T - c) * cs, cmax = std::min(m, (T - c + 1) * cs);
    int64_t rmin = cmin;                          // min row of the chunk's columns
    for (int64_t j = cmin; j < cmax; ++j)
      if (X.Up[j + 1] > X.Up[j]) rmin = std::min(rmin, X.Ui[X.Up[j]]);
    add(cmin, cmax, rmin, cmin, true);
  }
  hipStream_t st = h->stream;
  h->ch_data.free();
  h->ch_desc.free();
  h->ch_p.free();
  h->ch_q.free();
  HIPCHK(h->ch_data.upload(data.data(), data.size(), st));
  HIPCHK(h->ch_desc.upload(desc.data(), desc.size(), st));
  HIPCHK(h->ch_p.upload(X.p.data(), X.p.size(), st));
  HIPCHK(h->ch_q.upload(X.q.data(), X.q.size(), st));
  HIPCHK(hipStreamSynchronize(st));
  h->ch_T = T;
  h->ch_size = cs;
  h->ch_version = h->nfactor;
  return SMLU_OK;
}

// ldiv! (:286-342) through the chunked layout: wrk = (Rs.*b)[p]; lsolve!; rsolve!; x[q] = wrk.
// Device pointers; x may alias b.  Refills the chunks when the factors changed since the setup
// (the reference refills them in lu!, :265-276).
int smlu_chunked_ldiv_device(smlu_handle* h, const double* d_b, double* d_x) {
  if (!h || !d_b || !d_x) return fail(h, SMLU_ERR_ARG, "NULL argument");
  if (!h->have_numeric) return fail(h, SMLU_ERR_STATE, "no numeric factorization");
  if (h->ch_version != h->nfactor) {
    int rc = smlu_chunked_setup(h, h->ch_size);
    if (rc != SMLU_OK) return rc;
  }
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(after_caller(h));
  hipStream_t st = h->stream;
  const int64_t n = h->plan.n;
  double* w = h->wrk.p;
  HIPCHK(launch_perm_in(st, n, h->ch_p.p, h->Rs.p, d_b, w, 1, n, n));
  HIPCHK(launch_chunked_solve(st, false, h->ch_T, h->ch_desc.p, h->ch_data.p, w));
  HIPCHK(launch_chunked_solve(st, true, h->ch_T, h->ch_desc.p + h->ch_T, h->ch_data.p, w));
  HIPCHK(launch_perm_out(st, n, h->ch_q.p, w, d_x, 1, n, n));
  HIPCHK(hipStreamSynchronize(st));
  return SMLU_OK;
}

int smlu_chunked_ldiv(smlu_handle* h, const double* b, double* x) {
  if (!h || !b || !x) return fail(h, SMLU_ERR_ARG, "NULL argument");
  if (!h->have_numeric) return fail(h, SMLU_ERR_STATE, "no numeric factorization");
  HIPCHK(hipSetDevice(h->device));
  const int64_t n = h->plan.n;
  HIPCHK(hipMemcpyAsync(h->wrk2.p, b, sizeof(double) * n, hipMemcpyHostToDevice, h->stream));
  int rc = smlu_chunked_ldiv_device(h, h->wrk2.p, h->wrk2.p);
  if (rc != SMLU_OK) return rc;
  HIPCHK(hipMemcpyAsync(x, h->wrk2.p, sizeof(double) * n, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  return SMLU_OK;
}

