// factor.cpp — numeric refactorization: the captured factor segments, pivot status, the
// pivoting-mode decision, and the refactor entry points (lu! of src/SharedMemSparseLU.jl:245-279).
#include "handle.hpp"

static hipError_t run_launch(smlu_handle* h, const Launch& L, double diag_tol, double piv_tol, hipStream_t st) {
  switch (L.kind) {
    case K_EXTADD:
      return launch_assemble(st, L.cnt, h->xcols.p + L.off, h->xtasks.p, h->aents.p, h->sn.p, h->relmap.p,
                             h->A.p, h->Arow.p, h->Rs.p, h->store.p, h->scratch.p);
    case K_FRONT_LDS:
      return launch_front_small(st, (int)L.cnt, (int)L.aux, h->ilist.p + L.off, h->sn.p, h->chlist.p,
                                h->relmap.p, h->aents.p, h->A.p, h->Arow.p, h->Rs.p, h->store.p, h->scratch.p,
                                h->rowperm.p, h->info.p, h->growth.p, diag_tol, piv_tol);
    case K_STEPTRSM:
      return launch_step_trsm(st, (int)L.aux, h->ftiles.p + L.off, (int)L.cnt, L.nwg, h->ftiles.p + L.off2,
                              (int)L.cnt2, L.nwg2, L.step, h->ob, h->sn.p, h->store.p, h->scratch.p, h->info.p,
                              h->growth.p, piv_tol);
    case K_LASWP:
      return launch_laswp(st, L.nwg, h->stasks.p + L.off, (int)L.cnt, h->sn.p, h->store.p, h->scratch.p,
                          h->swaps.p, kSwapStride);
    case K_PANEL:
      return launch_panel1(st, (int)L.cnt, (int)L.aux, (int)L.nwg, (int)L.aux2, L.step,
                           h->ilist.p + L.off, h->sn.p,
                          h->store.p, h->scratch.p, h->rowperm.p, h->swaps.p, kSwapStride, h->info.p,
                          h->growth.p, diag_tol, (int)L.cnt2, h->tinv.p, (int)h->ob);
    case K_TRSMU:
      return launch_trsm_u(st, L.nwg, h->ftiles.p + L.off, (int)L.cnt, h->ob, (int)L.aux, h->sn.p,
                           h->store.p, h->scratch.p, h->swaps.p, kSwapStride);
    case K_GEMM:
    case K_GEMMU:
    case K_GEMMO:
    case K_GEMM22:
      return launch_gemm(st, L.nwg, h->gtasks.p + L.off, (int)L.cnt, (int)L.aux, 0);
    case K_TRSML:
      return launch_gemm_g(st, L.nwg, h->gtasks.p + L.off, (int)L.cnt, (int)L.aux, 0, h->info.p,
                           h->growth.p, piv_tol);
    case K_UROWS:
      return launch_urows(st, (int)L.cnt, h->urtasks.p + L.off, h->sn.p, h->store.p, h->tinv.p);
    case K_TRIINV:
      return launch_tri_inv(st, (int)L.cnt, L.step, h->ilist.p + L.off, h->sn.p, h->store.p, h->scratch.p,
                            h->tinv.p);
  }
  return hipErrorInvalidValue;
}

// All device work of one numeric refactorization, in stream order (captured into a graph).
// Segment `seg` of one numeric refactorization (launches between two exchange points; the
// whole refactor is the single segment 0 on one GPU), in stream order.
static int enqueue_factor(smlu_handle* h, Timer& tm, bool dbg, int seg) {
  Plan& P = h->plan;
  hipStream_t st = h->stream;
  const size_t lo = h->fac_seg[seg];
  const size_t hi = (size_t)seg + 1 < h->fac_seg.size() ? h->fac_seg[seg + 1] : h->fac.size();
  double diag_tol = P.given_order ? 0.0 : h->opts.diag_pivot_tol;
  double piv_tol = h->opts.pivot_tol;
  if (seg > 0) goto launches;
  // info words and growth cleared, identity (local) row permutation (fronts overwrite their part):
  // one kernel, so that the captured graph holds kernel nodes only
  HIPCHK(launch_factor_reset(st, h->nnodes, h->info.p, h->growth.p, P.n, h->rowperm.p, h->rowperm0.p));
  if (!h->given_Rs) {
    if (h->opts.scale) HIPCHK(launch_rowscale(st, P.n, h->Arowptr.p, h->Arow_ent.p, h->A.p, h->Rs.p));
    else HIPCHK(launch_fill(st, P.n, h->Rs.p, 1.0));
  }
  // A given (p, q) order means "no pivoting on top": only a zero diagonal moves (diag_tol 0).
launches:
  // the size classes of one level's small fronts (K_FRONT_LDS launches of one overlap group)
  // alternate between the handle's stream and its side stream: a fork event ahead of the group,
  // a join event after its last launch
  // (profile mode: a group is timed once, on the main stream from before the fork to after the
  // join, so the overlapped branches are not counted twice)
  auto group = [&](size_t i) { return h->fac[i].kind == K_FRONT_LDS ? h->fac[i].aux2 : 0; };
  int gi = 0;   // index of the current launch inside its group
  hipEvent_t gstop = nullptr;
  for (size_t li = lo; li < hi; ++li) {
    const Launch& L = h->fac[li];
    const int64_t g = group(li);
    const bool cont = g > 0 && li > lo && group(li - 1) == g;
    const bool more = g > 0 && li + 1 < hi && group(li + 1) == g;
    gi = cont ? gi + 1 : 0;
    const bool grouped = cont || more;
    // fork: the side stream starts after everything before the group (recorded ahead of the
    // group's first launch, waited on by the side stream before its first)
    if (gi == 0 && more) {
      HIPCHK(tm.begin(L.kind, &gstop, st));
      HIPCHK(hipEventRecord(h->fork_ev, st));
    }
    if (gi == 1) HIPCHK(hipStreamWaitEvent(h->side, h->fork_ev, 0));
    hipStream_t ls = (gi & 1) ? h->side : st;
    hipEvent_t stop = nullptr;
    if (!grouped) HIPCHK(tm.begin(L.kind, &stop, ls));
    hipError_t e = run_launch(h, L, diag_tol, piv_tol, ls);
    if (e == hipSuccess && dbg) e = hipStreamSynchronize(ls);
    if (e != hipSuccess) {
      if (gi >= 1) {   // the side stream's branch is joined on the error path too (capture stays valid)
        (void)hipEventRecord(h->join_ev, h->side);
        (void)hipStreamWaitEvent(st, h->join_ev, 0);
      }
      char buf[256];
      std::snprintf(buf, sizeof buf, "HIP error '%s' in launch kind=%d step=%d off=%lld cnt=%lld nwg=%lld aux=%lld aux2=%lld",
                    hipGetErrorString(e), L.kind, L.step, (long long)L.off, (long long)L.cnt,
                    (long long)L.nwg, (long long)L.aux, (long long)L.aux2);
      return fail(h, SMLU_ERR_HIP, buf);
    }
    if (!grouped) HIPCHK(tm.end(stop));
    if (gi >= 1 && !more) {   // join: the main stream continues after both branches
      HIPCHK(hipEventRecord(h->join_ev, h->side));
      HIPCHK(hipStreamWaitEvent(st, h->join_ev, 0));
      tm.st = st;
      HIPCHK(tm.end(gstop));
      gstop = nullptr;
    }
  }
  return SMLU_OK;
}

// Run factor segment `seg`: captured once into a hipGraph and replayed (the first
// factorization runs eagerly).
static int factor_segment(smlu_handle* h, Timer& tm, int seg) {
  hipStream_t st = h->stream;
  const Tune tn = tune();
  const bool dbg = tn.debug_sync, nograph = tn.no_graph;
  const int prof = h->opts.profile ? 1 : 0;
  const size_t nseg = h->fac_seg.size();
  if (h->fac_execs.size() != nseg || (seg == 0 && h->fac_exec_profile != prof)) {
    for (auto& g : h->fac_execs)
      if (g) (void)hipGraphExecDestroy(g);
    h->fac_execs.assign(nseg, nullptr);
    h->seg_events.assign(nseg, {0, 0});
  }
  bool use_graph = !dbg && !nograph && !h->graph_failed && h->have_numeric;  // first run eager
  if (use_graph && !h->fac_execs[seg]) {
    hipGraph_t g = nullptr;
    const size_t ev0 = tm.used;
    HIPCHK(hipStreamBeginCapture(st, hipStreamCaptureModeRelaxed));
    int rc = enqueue_factor(h, tm, false, seg);
    hipError_t ec = hipStreamEndCapture(st, &g);
    if (rc == SMLU_OK && ec == hipSuccess && g) ec = hipGraphInstantiate(&h->fac_execs[seg], g, nullptr, nullptr, 0);
    if (g) (void)hipGraphDestroy(g);
    if (rc != SMLU_OK || ec != hipSuccess || !h->fac_execs[seg]) {
      (void)hipGetLastError();
      h->graph_failed = true;   // fall back to eager launches
      h->fac_execs[seg] = nullptr;
      use_graph = false;
      tm.used = ev0;
    } else {
      h->fac_exec_profile = prof;
      h->seg_events[seg] = {ev0, tm.used - ev0};
    }
  }
  if (use_graph) {
    tm.used = h->seg_events[seg].first + h->seg_events[seg].second;
    HIPCHK(hipGraphLaunch(h->fac_execs[seg], st));
    return SMLU_OK;
  }
  return enqueue_factor(h, tm, dbg, seg);
}

// Status words for the host (factor pivot status, dominance flags, sweep timeouts) travel as one
// 64-byte record written by k_status behind the work on the stream and stamped at both ends with a
// per-read sequence number; the host takes a copy only when both stamps match and copies again
// otherwise.  (Observed on the MI355X box: a 1.4 MB device-to-host copy of the per-front info words
// into pinned memory, issued right after a graph replay, once delivered foreign data -- an array of
// device pointers -- which read as a weak pivot in every front and forced a re-pivoting refactor;
// nothing in a factorization's status is taken on trust since.)
int read_status(smlu_handle* h, const int32_t* info, int64_t nnodes, const int32_t* words, int nwords,
                long long out[16]) {
  hipStream_t st = h->stream;
  const long long seq = ++h->rb_seq;
  HIPCHK(launch_status(st, info, nnodes, info ? h->sn.p : nullptr, words, nwords, h->rb.p, seq));
  HIPCHK(hipStreamSynchronize(st));
  for (int attempt = 0; attempt < 4; ++attempt) {
    HIPCHK(hipMemcpy(out, h->rb.p, 16 * sizeof(long long), hipMemcpyDeviceToHost));
    if (out[0] == seq && out[15] == seq) return SMLU_OK;
    ++h->status_copy_retries;   // counted (smlu_stat "status_copy_retries"): the tests require 0
  }
  return fail(h, SMLU_ERR_HIP, "status record read back with a wrong sequence stamp (device-to-host copy)");
}

// After the last segment: pivot status of this rank's fronts.
static int finish_factor(smlu_handle* h, Timer& tm, std::chrono::steady_clock::time_point t0) {
  Plan& P = h->plan;
  long long rec[16];
  // words: the growth maximum (growth[0]) and the dominance flags of the values (growth[1], two
  // int32: by columns, by rows; written by k_dominance ahead of the factorization when the
  // pivoting mode is re-decided) -- one record, one synchronisation per factorization
  int rs = read_status(h, h->info.p, h->nnodes, reinterpret_cast<const int32_t*>(h->growth.p), 4, rec);
  if (rs != SMLU_OK) return rs;
  h->dom_words = rec[7];
  if (rec[10] > 0) {   // an info word no factor kernel writes: never read as a pivot status
    h->bad_info_node = rec[8];
    h->bad_info_word = (int32_t)rec[9];
    h->bad_info_count += rec[10];
    return fail(h, SMLU_ERR_STATE, "factorization status: " + std::to_string(rec[10]) +
                " front info words outside the legal code set (first: node " + std::to_string(rec[8]) +
                ", word " + std::to_string(rec[9]) + ")");
  }
  tm.collect();
  h->refactor_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  double g;
  std::memcpy(&g, &rec[6], sizeof g);
  h->growth_max = g;
  h->have_numeric = true;
  ++h->nfactor;
  h->weak = rec[1];
  h->errcol = -1;
  h->flag_node = rec[4];
  h->flag_info = (int32_t)rec[5];
  int rc = SMLU_OK;
  if (rec[2] >= 0) {
    const int32_t v = (int32_t)rec[3];
    rc = SMLU_SINGULAR;
    h->errcol = P.s_first[h->node_front[rec[2]]] + ((v >> 2) > 0 ? (v >> 2) - 1 : 0);
  }
  if (h->nranks > 1) {   // the pivot status of the whole partition, on every rank
    double red[3] = {rc == SMLU_SINGULAR ? 1.0 : 0.0, (double)h->errcol, (double)h->weak};
    if (h->tr.allreduce_max(h->tr.ctx, red, 3) != 0) return fail(h, SMLU_ERR_HIP, "transport allreduce failed");
    rc = red[0] > 0 ? SMLU_SINGULAR : SMLU_OK;
    h->errcol = (int64_t)red[1];
    h->weak = (int64_t)red[2];
  }
  if (rc == SMLU_SINGULAR) h->err = "matrix is singular (zero pivot column)";
  return rc;
}

// One communication step: pack copies, the transfer through the transport, unpack copies.
// Device-memory transports (RCCL) are enqueued on the stream; host-memory ones go through the
// pinned staging buffers after a stream synchronisation.
static int run_factor_once(smlu_handle* h) {
  HIPCHK(hipSetDevice(h->device));
  auto t0 = std::chrono::steady_clock::now();
  for (auto& v : h->kind_ms) v = 0;
  h->comm_sent_fac = h->comm_recv_fac = 0;
  Timer tm(h);
  for (size_t seg = 0; seg < h->fac_seg.size(); ++seg) {
    if (seg > 0) {
      int rc = exec_comm(h, h->fac_comm[seg - 1]);
      if (rc != SMLU_OK) return rc;
    }
    int rc = factor_segment(h, tm, (int)seg);
    if (rc != SMLU_OK) return rc;
  }
  return finish_factor(h, tm, t0);
}

static int apply_dominance(smlu_handle* h, bool dom, bool* rebuilt);
static int launch_device_dominance(smlu_handle* h);

// One factorization of the values in h->A with the re-pivoting fallback.  redecide: the pivoting
// mode is re-decided for these values without a synchronisation of its own:
// k_dominance runs ahead of the factorization, which goes on in the current mode, and its flags
// come back in the factorization's status record; only when they call for another mode (rare:
// the values changed between dominant and non-dominant, or a re-pivoted handle sees dominant
// values again) is the schedule rebuilt and the same values factored again in that mode.
int run_factor(smlu_handle* h, bool redecide) {
  if (redecide) {
    int rc = launch_device_dominance(h);
    if (rc != SMLU_OK) return rc;
  }
  int rc = run_factor_once(h);
  if (rc < 0) return rc;
  if (redecide) {
    const bool dom = (h->dom_words & 0xffffffffll) != 0 || (h->dom_words >> 32) != 0;
    bool rebuilt = false;
    int r2 = apply_dominance(h, dom, &rebuilt);
    if (r2 != SMLU_OK) return r2;
    if (rebuilt) {
      ++h->mode_refactors;
      return run_factor(h, false);
    }
  }
  const bool off = tune().no_repivot;   // test knob
  if ((rc == SMLU_SINGULAR || h->weak > 0) && h->pivmode == 0 && !off && has_tile_fronts(h) &&
      h->opts.pivot_tol > 0 && !h->plan.given_order && h->nranks == 1) {
    h->repivot_node = h->flag_node;
    h->repivot_info = h->flag_info;
    h->repivot_sn = h->flag_node >= 0 && h->flag_node < (int64_t)h->hsn.size() ? h->hsn[h->flag_node] : SNode{};
    h->repivot_growth = h->growth_max;
    h->pivmode = 1;
    int r2 = rebuild_schedule(h);
    if (r2 != SMLU_OK) return r2;
    ++h->repivots;
    rc = run_factor_once(h);
  }
  return rc;
}


// Pivoting mode per refactor: dominant values take the diagonal-tile path for
// every blocked front; a handle left in full-candidate mode by a re-pivoting refactor returns to
// the fast schedule once the values are dominant again.  The ranks of a partitioned handle agree
// on the decision (any rank seeing non-dominant values makes it non-dominant for all): a rebuild
// on only some ranks would split the collective schedule.
static int apply_dominance(smlu_handle* h, bool dom, bool* rebuilt) {
  *rebuilt = false;
  if (h->nranks > 1) {
    double nd = dom ? 0.0 : 1.0;
    if (h->tr.allreduce_max(h->tr.ctx, &nd, 1) != 0) return fail(h, SMLU_ERR_HIP, "transport allreduce failed (dominance)");
    dom = nd == 0.0;
  }
  bool changed = false;
  if (dom != h->dominant) {
    h->dominant = dom;
    changed = h->pivmode == 0;
  }
  if (dom && h->pivmode == 1) {
    h->pivmode = 0;
    changed = true;
  }
  *rebuilt = changed;
  return changed ? rebuild_schedule(h) : SMLU_OK;
}

// The dominance test of the values in HBM (k_dominance: one thread per column and row, the host
// diagonally_dominant()'s summation order), flags into growth[1] for finish_factor's record.
static int launch_device_dominance(smlu_handle* h) {
  const Plan& P = h->plan;
  hipStream_t st = h->stream;
  if (!h->Acolp.p) HIPCHK(h->Acolp.upload(P.Acolptr.data(), P.Acolptr.size(), st));
  int rc = ensure_residual(h);   // the column of every A entry
  if (rc != SMLU_OK) return rc;
  HIPCHK(launch_dominance(st, P.n, h->Acolp.p, h->Arow.p, h->Arowptr.p, h->Arow_ent.p, h->Acol.p, h->A.p,
                          reinterpret_cast<int32_t*>(h->growth.p + 1)));
  return SMLU_OK;
}

// lu! on the values already in h->A: the factorization with the pivoting mode re-decided for
// these values (above) and the re-pivoting fallback.
int refactor_resident(smlu_handle* h) {
  return run_factor(h, !h->plan.given_order && !h->plan.matched);
}

int smlu_refactor(smlu_handle* h, const double* nzval) {
  if (!h || !nzval) return fail(h, SMLU_ERR_ARG, "NULL argument");
  HIPCHK(hipSetDevice(h->device));
  // the values' upload, then the device path (dominance on the device, no host scan of the values)
  HIPCHK(hipMemcpyAsync(h->A.p, nzval, sizeof(double) * h->plan.nnzA, hipMemcpyHostToDevice, h->stream));
  return refactor_resident(h);   // collective on a partitioned handle
}

// Device entry points read caller memory (values, right-hand sides) on the handle's own stream:
// order that stream after the work the caller has enqueued on its stream so far (an event, no
// host wait).  Outputs are complete when an entry point returns (it synchronises its stream).
hipError_t after_caller(smlu_handle* h) {
  if (!h->ev_caller) {
    hipError_t e = hipEventCreateWithFlags(&h->ev_caller, hipEventDisableTiming);
    if (e != hipSuccess) return e;
  }
  hipError_t e = hipEventRecord(h->ev_caller, h->caller);
  return e != hipSuccess ? e : hipStreamWaitEvent(h->stream, h->ev_caller, 0);
}

// Dev (tools/determinism.py, not in smlu.h): per supernode of a one-GPU handle, a hash of its
// factor values and one of its row permutation, out[2s], out[2s+1] (2 * nsuper entries).
int smlu_dev_front_hash(smlu_handle* h, unsigned long long* out) {
  if (!h || !out) return fail(h, SMLU_ERR_ARG, "NULL argument");
  if (h->nranks > 1) return fail(h, SMLU_ERR_STATE, "one-GPU handles only");
  const int64_t ns = h->plan.nsup;
  DBuf<unsigned long long> d;
  HIPCHK(d.alloc((size_t)std::max<int64_t>(2 * ns, 1)));
  HIPCHK(launch_front_hash(h->stream, ns, h->sn.p, h->store.p, h->rowperm.p, d.p));
  HIPCHK(hipStreamSynchronize(h->stream));
  hipError_t e = hipMemcpy(out, d.p, sizeof(unsigned long long) * 2 * ns, hipMemcpyDeviceToHost);
  d.free();
  HIPCHK(e);
  return SMLU_OK;
}

// Dev (tools/determinism.py, not in smlu.h): the factor values of supernode s as stored, L panel
// (M x ns, ld M) then U12 (ns x nu, ld ns); out holds M*ns + ns*nu doubles.
int smlu_dev_front_values(smlu_handle* h, int64_t s, double* out) {
  if (!h || !out || s < 0 || s >= h->plan.nsup) return fail(h, SMLU_ERR_ARG, "invalid arguments");
  if (h->nranks > 1) return fail(h, SMLU_ERR_STATE, "one-GPU handles only");
  const SNode& r = h->hsn[s];
  const int64_t M = (int64_t)r.ns + r.nu;
  HIPCHK(hipStreamSynchronize(h->stream));
  HIPCHK(hipMemcpy(out, h->store.p + r.Loff, sizeof(double) * M * r.ns, hipMemcpyDeviceToHost));
  if (r.nu > 0)
    HIPCHK(hipMemcpy(out + M * r.ns, h->store.p + r.Uoff, sizeof(double) * r.ns * r.nu, hipMemcpyDeviceToHost));
  return SMLU_OK;
}

// Dev (tools/determinism.py, not in smlu.h): doubles [off, off+cnt) of the factor store (which 0)
// or of the front scratch (which 1) to host memory; cnt < 0 returns the buffer's length in *len.
int smlu_dev_copy(smlu_handle* h, int which, int64_t off, int64_t cnt, double* out, int64_t* len) {
  if (!h || which < 0 || which > 1) return fail(h, SMLU_ERR_ARG, "invalid arguments");
  const DBuf<double>& b = which == 0 ? h->store : h->scratch;
  if (cnt < 0) {
    if (len) *len = (int64_t)b.n;
    return SMLU_OK;
  }
  if (!out || off < 0 || off + cnt > (int64_t)b.n) return fail(h, SMLU_ERR_ARG, "range outside the buffer");
  HIPCHK(hipStreamSynchronize(h->stream));
  HIPCHK(hipMemcpy(out, b.p + off, sizeof(double) * cnt, hipMemcpyDeviceToHost));
  return SMLU_OK;
}

// Dev (not in smlu.h): per supernode Loff, Uoff, Foff (-1: no F22) and M, 4 * nsuper entries.
int smlu_dev_front_offsets(smlu_handle* h, int64_t* out) {
  if (!h || !out) return fail(h, SMLU_ERR_ARG, "NULL argument");
  for (int64_t s = 0; s < h->plan.nsup; ++s) {
    const SNode& r = h->hsn[s];
    out[4 * s] = r.Loff;
    out[4 * s + 1] = r.Uoff;
    out[4 * s + 2] = r.Foff;
    out[4 * s + 3] = (int64_t)r.ns + r.nu;
  }
  return SMLU_OK;
}

int smlu_set_stream(smlu_handle* h, void* stream) {
  if (!h) return fail(h, SMLU_ERR_ARG, "NULL handle");
  h->caller = reinterpret_cast<hipStream_t>(stream);
  return SMLU_OK;
}

int smlu_refactor_device(smlu_handle* h, const double* d_nzval) {
  if (!h || !d_nzval) return fail(h, SMLU_ERR_ARG, "NULL argument");
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(after_caller(h));
  if (d_nzval != h->A.p)
    HIPCHK(hipMemcpyAsync(h->A.p, d_nzval, sizeof(double) * h->plan.nnzA, hipMemcpyDeviceToDevice, h->stream));
  return refactor_resident(h);
}

int smlu_refactor_csc(smlu_handle* h, int64_t n, const int64_t* colptr, const int64_t* rowval,
                      const double* nzval) {
  if (!h || !colptr || !rowval || !nzval) return fail(h, SMLU_ERR_ARG, "NULL argument");
  if (h->zc) return fail(h, SMLU_ERR_ARG, "complex handle: use smlu_refactor_csc_z");
  return refactor_csc_impl(h, n, colptr, rowval, nzval, nullptr);
}


int refactor_csc_impl(smlu_handle* h, int64_t n, const int64_t* colptr, const int64_t* rowval,
                      const double* nzval, const std::vector<int64_t>* preorder) {
  if (h->nranks > 1) return fail(h, SMLU_ERR_STATE, "partitioned handle: create a new one for a new pattern");
  const Plan& P = h->plan;
  int base = h->opts.index_base;
  bool same = (n == P.n);
  for (int64_t j = 0; same && j <= n; ++j) same = (colptr[j] - base == P.Acolptr[j]);
  for (int64_t e = 0; same && e < P.nnzA; ++e) same = (rowval[e] - base == P.Arow[e]);
  if (same) return smlu_refactor(h, nzval);
  // pattern changed: the reference re-chunks and re-allocates (src/SharedMemSparseLU.jl:265-273);
  // here: re-analysis and re-allocation in place, keeping the options and the stream.
  h->release_buffers();
  h->have_numeric = false;
  h->given_Rs = false;
  // the caller's UMFPACK pattern (smlu_create_with_pivots) belongs to the old (p, q) and the old
  // pattern of A: the new factors are exported on their own structural pattern
  h->given_pattern = false;
  h->gLp.clear();
  h->gLi.clear();
  h->gUp.clear();
  h->gUi.clear();
  h->pattern_dropped = 0;
  h->plan = Plan();
  std::string e;
  try {
    std::vector<int64_t> match = diagonal_match(n, colptr, rowval, nzval, base);
    PlanOptions po = plan_opts(h->opts);
    if (preorder) po.preorder = *preorder;
    e = h->plan.build(n, colptr, rowval, base, po, nullptr, nullptr,
                      match.empty() ? nullptr : match.data());
  } catch (const std::bad_alloc&) {
    return fail(h, SMLU_ERR_ALLOC, "host allocation failed during analysis");
  }
  if (!e.empty()) return fail(h, SMLU_ERR_ARG, e);
  h->dominant = !h->plan.matched && diagonally_dominant(n, colptr, rowval, nzval, base);
  h->pivmode = 0;
  h->cpair = preorder != nullptr && !h->plan.matched;
  int rc = setup_device(h);
  if (rc != SMLU_OK) return rc;
  HIPCHK(hipMemcpyAsync(h->A.p, nzval, sizeof(double) * h->plan.nnzA, hipMemcpyHostToDevice, h->stream));
  return run_factor(h);
}


