// dist.cpp — multi-GPU: the built-in RCCL transport, the exchange / broadcast steps of a
// partitioned schedule, and the partition entry points (smlu_dist_*, smlu_plan_partition / _project).
#include "handle.hpp"

namespace smlu {

RcclApi* rccl_api() {
  static RcclApi api;
  static bool tried = false;
  if (tried) return api.lib ? &api : nullptr;
  tried = true;
  void* l = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
  if (!l) l = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
  if (!l) return nullptr;
  bool ok = true;
  auto sym = [&](const char* n) {
    void* f = dlsym(l, n);
    ok = ok && f != nullptr;
    return f;
  };
  api.GetUniqueId = (decltype(api.GetUniqueId))sym("ncclGetUniqueId");
  api.CommInitRank = (decltype(api.CommInitRank))sym("ncclCommInitRank");
  api.CommDestroy = (decltype(api.CommDestroy))sym("ncclCommDestroy");
  api.Send = (decltype(api.Send))sym("ncclSend");
  api.Recv = (decltype(api.Recv))sym("ncclRecv");
  api.GroupStart = (decltype(api.GroupStart))sym("ncclGroupStart");
  api.GroupEnd = (decltype(api.GroupEnd))sym("ncclGroupEnd");
  api.AllReduce = (decltype(api.AllReduce))sym("ncclAllReduce");
  api.CommCount = (decltype(api.CommCount))sym("ncclCommCount");
  if (!ok) return nullptr;
  api.lib = l;
  return &api;
}

int rccl_exchange(void* ctx, int32_t npeer, const int32_t* peer, void* const* sbuf, const int64_t* sbytes,
                  void* const* rbuf, const int64_t* rbytes, void* stream) {
  RcclApi* R = rccl_api();
  auto* S = static_cast<RcclState*>(ctx);
  hipStream_t st = (hipStream_t)stream;
  if (R->GroupStart() != ncclSuccess) return 1;
  int rc = 0;   // on a failed send/recv the group is still closed, so the communicator stays usable
  for (int32_t i = 0; i < npeer && rc == 0; ++i) {
    if (sbytes[i] > 0 && R->Send(sbuf[i], (size_t)sbytes[i], ncclUint8, peer[i], S->comm, st) != ncclSuccess) rc = 2;
    else if (rbytes[i] > 0 && R->Recv(rbuf[i], (size_t)rbytes[i], ncclUint8, peer[i], S->comm, st) != ncclSuccess) rc = 3;
  }
  const bool ended = R->GroupEnd() == ncclSuccess;
  return rc != 0 ? rc : ended ? 0 : 4;
}

// broadcast inside a rank group as root -> member sends (the group is a subset of the ranks)
int rccl_bcast(void* ctx, void* buf, int64_t bytes, int32_t root, int32_t gsize, const int32_t* group, void* stream) {
  RcclApi* R = rccl_api();
  auto* S = static_cast<RcclState*>(ctx);
  hipStream_t st = (hipStream_t)stream;
  if (bytes <= 0) return 0;
  if (R->GroupStart() != ncclSuccess) return 1;
  int rc = 0;   // GroupEnd runs on the error path too
  if (S->rank == root) {
    for (int32_t i = 0; i < gsize && rc == 0; ++i)
      if (group[i] != root && R->Send(buf, (size_t)bytes, ncclUint8, group[i], S->comm, st) != ncclSuccess) rc = 2;
  } else if (R->Recv(buf, (size_t)bytes, ncclUint8, root, S->comm, st) != ncclSuccess) {
    rc = 3;
  }
  const bool ended = R->GroupEnd() == ncclSuccess;
  return rc != 0 ? rc : ended ? 0 : 4;
}

int rccl_allreduce_max(void* ctx, double* buf, int32_t count) {
  RcclApi* R = rccl_api();
  auto* S = static_cast<RcclState*>(ctx);
  if (count > 8) return 1;
  if (hipMemcpyAsync(S->dbuf, buf, sizeof(double) * count, hipMemcpyHostToDevice, S->stream) != hipSuccess) return 2;
  if (R->AllReduce(S->dbuf, S->dbuf, (size_t)count, ncclFloat64, ncclMax, S->comm, S->stream) != ncclSuccess) return 3;
  if (hipMemcpyAsync(buf, S->dbuf, sizeof(double) * count, hipMemcpyDeviceToHost, S->stream) != hipSuccess) return 4;
  return hipStreamSynchronize(S->stream) == hipSuccess ? 0 : 5;
}

}  // namespace smlu

int exec_comm(smlu_handle* h, int id) {
  CommOp& op = h->comm[id];
  hipStream_t st = h->stream;
  HIPCHK(launch_segcopy(st, h->segdesc.p + op.pack0, (int64_t)op.pack.size()));
  char* base[10] = {(char*)h->store.p, (char*)h->scratch.p, (char*)h->vbuf.p, (char*)h->wrk.p,
                    (char*)h->stage_s.p, (char*)h->stage_r.p, (char*)h->bcbuf.p, (char*)h->tinv.p,
                    (char*)h->swaps.p, (char*)h->rowperm.p};
  const bool dev = h->tr.device_memory != 0;
  int e = 0;
  if (op.type == 1) {
    char* buf = base[op.bbase];
    if (dev) {
      e = h->tr.bcast(h->tr.ctx, buf, op.bytes, op.root, (int32_t)op.grp.size(), op.grp.data(), (void*)st);
    } else {
      char* hb = h->rank == op.root ? h->hstage_s : h->hstage_r;
      if (h->rank == op.root) HIPCHK(hipMemcpyAsync(hb, buf, op.bytes, hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));
      e = h->tr.bcast(h->tr.ctx, hb, op.bytes, op.root, (int32_t)op.grp.size(), op.grp.data(), nullptr);
      if (e == 0 && h->rank != op.root) HIPCHK(hipMemcpyAsync(buf, hb, op.bytes, hipMemcpyHostToDevice, st));
    }
  } else {
    const int np = (int)op.peer.size();
    std::vector<void*> sb(np), rb(np);
    if (dev) {
      for (int i = 0; i < np; ++i) {
        sb[i] = base[op.sbase[i]] + op.soff[i];
        rb[i] = base[op.rbase[i]] + op.roff[i];
      }
      e = h->tr.exchange(h->tr.ctx, np, op.peer.data(), sb.data(), op.sbytes.data(), rb.data(), op.rbytes.data(),
                         (void*)st);
    } else {
      // host staging: sends packed side by side, receives side by side
      int64_t so = 0, ro = 0;
      for (int i = 0; i < np; ++i) {
        if (op.sbytes[i] > 0)
          HIPCHK(hipMemcpyAsync(h->hstage_s + so, base[op.sbase[i]] + op.soff[i], op.sbytes[i], hipMemcpyDeviceToHost, st));
        sb[i] = h->hstage_s + so;
        rb[i] = h->hstage_r + ro;
        so += op.sbytes[i];
        ro += op.rbytes[i];
      }
      HIPCHK(hipStreamSynchronize(st));
      e = h->tr.exchange(h->tr.ctx, np, op.peer.data(), sb.data(), op.sbytes.data(), rb.data(), op.rbytes.data(),
                         nullptr);
      for (int i = 0; i < np && e == 0; ++i)
        if (op.rbytes[i] > 0)
          HIPCHK(hipMemcpyAsync(base[op.rbase[i]] + op.roff[i], rb[i], op.rbytes[i], hipMemcpyHostToDevice, st));
    }
  }
  if (e != 0) return fail(h, SMLU_ERR_HIP, "transport error " + std::to_string(e) + " in communication step");
  {   // bytes moved by this rank (bench.py: comm_bytes per rank)
    double sent = 0, recv = 0;
    if (op.type == 1) {
      if (h->rank == op.root) sent = (double)op.bytes * (double)(op.grp.size() - 1);
      else recv = (double)op.bytes;
    } else {
      for (size_t i = 0; i < op.peer.size(); ++i) {
        sent += (double)op.sbytes[i];
        recv += (double)op.rbytes[i];
      }
    }
    h->comm_sent += sent;
    h->comm_recv += recv;
    h->comm_sent_fac += sent;
    h->comm_recv_fac += recv;
    ++h->comm_calls;
  }
  HIPCHK(launch_segcopy(st, h->segdesc.p + op.unpack0, (int64_t)op.unpack.size()));
  return SMLU_OK;
}

// ---- multi-GPU partition (one process per GPU; collective; transport supplied or RCCL) ----
int smlu_dist_create(int64_t n, const int64_t* colptr, const int64_t* rowval, const double* nzval,
                     const smlu_opts* opts, int32_t rank, int32_t nranks, const smlu_transport* tr,
                     smlu_handle** out) {
  if (nranks < 1 || rank < 0 || rank >= nranks) return fail(nullptr, SMLU_ERR_ARG, "bad rank/nranks");
  if (nranks > 1 && (!tr || !tr->exchange || !tr->bcast || !tr->allreduce_max))
    return fail(nullptr, SMLU_ERR_ARG, "a partitioned handle needs a complete transport");
  return create_impl(n, colptr, rowval, nzval, nullptr, nullptr, nullptr, opts, out, rank, nranks, tr);
}

int smlu_rccl_unique_id(uint8_t id[128]) {
  if (!id) return fail(nullptr, SMLU_ERR_ARG, "NULL id");
  RcclApi* R = rccl_api();
  if (!R) return fail(nullptr, SMLU_ERR_HIP, "librccl not loadable");
  ncclUniqueId u;
  if (R->GetUniqueId(&u) != ncclSuccess) return fail(nullptr, SMLU_ERR_HIP, "ncclGetUniqueId failed");
  std::memcpy(id, &u, sizeof(u) < 128 ? sizeof(u) : 128);
  return SMLU_OK;
}

int smlu_dist_create_rccl(int64_t n, const int64_t* colptr, const int64_t* rowval, const double* nzval,
                          const smlu_opts* opts, int32_t rank, int32_t nranks, const uint8_t id[128],
                          smlu_handle** out) {
  if (!id || nranks < 1 || rank < 0 || rank >= nranks) return fail(nullptr, SMLU_ERR_ARG, "bad arguments");
  RcclApi* R = rccl_api();
  if (!R) return fail(nullptr, SMLU_ERR_HIP, "librccl not loadable");
  const int dev = opts ? opts->device : 0;
  if (hipSetDevice(dev) != hipSuccess) return fail(nullptr, SMLU_ERR_NODEVICE, "hipSetDevice failed");
  auto* st = new (std::nothrow) RcclState();
  if (!st) return fail(nullptr, SMLU_ERR_ALLOC, "allocation failed");
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof(u) < 128 ? sizeof(u) : 128);
  if (R->CommInitRank(&st->comm, nranks, u, rank) != ncclSuccess) {
    delete st;
    return fail(nullptr, SMLU_ERR_HIP, "ncclCommInitRank failed");
  }
  st->rank = rank;
  if (R->CommCount(st->comm, &st->comm_count) != ncclSuccess || st->comm_count != nranks) {
    (void)R->CommDestroy(st->comm);
    delete st;
    return fail(nullptr, SMLU_ERR_HIP, "ncclCommCount does not report the requested rank count");
  }
  smlu_transport tr{};
  tr.ctx = st;
  tr.device_memory = 1;
  tr.exchange = rccl_exchange;
  tr.bcast = rccl_bcast;
  tr.allreduce_max = rccl_allreduce_max;
  return create_impl(n, colptr, rowval, nzval, nullptr, nullptr, nullptr, opts, out, rank, nranks, &tr, st);
}

int smlu_plan_partition(const smlu_plan* plan, int32_t nparts, int32_t* owner, int64_t* nshared) {
  if (!plan || nparts < 1) return fail(nullptr, SMLU_ERR_ARG, "invalid arguments");
  Plan P = plan->plan;   // copy: the partition is a query
  P.compute_owners(nparts, kOBDefault);
  int64_t k = 0;
  for (int64_t s = 0; s < P.nsup; ++s) {
    if (owner) owner[s] = P.owner[s];
    if (P.dist(s)) ++k;
  }
  if (nshared) *nshared = k;
  return SMLU_OK;
}

int smlu_plan_rank_memory(const smlu_plan* plan, int32_t nparts, int32_t rank, double* store_bytes,
                          double* scratch_bytes, double* stage_bytes) {
  if (!plan || nparts < 1 || rank < 0 || rank >= nparts) return fail(nullptr, SMLU_ERR_ARG, "invalid arguments");
  Plan P = plan->plan;
  P.compute_owners(nparts, kOBDefault);
  RankLayout Y;
  if (nparts > 1) {
    rank_layout(P, rank, Y);
  } else {
    Y.store_size = P.factor_size;
    Y.scratch_size = P.scratch_size;
  }
  if (store_bytes) *store_bytes = 8.0 * (double)Y.store_size;
  if (scratch_bytes) *scratch_bytes = 8.0 * (double)Y.scratch_size;
  if (stage_bytes) *stage_bytes = 8.0 * (double)Y.stage_size * (nparts > 1 ? 3 : 0);   // block buffer + 2 staging
  return SMLU_OK;
}

double smlu_plan_project(const smlu_plan* plan, int32_t nparts, double tflops, double gbs, double lat_us,
                         double* t1) {
  if (!plan || nparts < 1) return std::numeric_limits<double>::quiet_NaN();
  Plan P = plan->plan;
  P.compute_owners(nparts, kOBDefault);
  return project_partition(P, tflops, gbs, lat_us, t1);
}


int smlu_plan_rank_schedule(const smlu_plan* plan, int32_t nparts, int32_t rank, int64_t* ops, int64_t cap,
                            int64_t* len, double bytes[5], int64_t counts[3]) {
  if (!plan || !len || nparts < 1 || rank < 0 || rank >= nparts || (ops && cap < 0))
    return fail(nullptr, SMLU_ERR_ARG, "invalid arguments");
  std::unique_ptr<smlu_handle> h(new (std::nothrow) smlu_handle());
  if (!h) return fail(nullptr, SMLU_ERR_ALLOC, "allocation failed");
  smlu_default_opts(&h->opts);
  h->opts.index_base = 0;
  int rc = SMLU_OK;
  try {
    h->plan = plan->plan;   // copy: the partition is this query's
    h->rank = rank;
    h->nranks = nparts;
    h->dominant = true;     // the collective schedule does not depend on the pivoting mode
    if (nparts > 1) {
      if (tune().ob > 0) h->ob = tune().ob;
      h->plan.compute_owners(nparts, h->ob);
    }
    rc = build_schedule_host(h.get());
  } catch (const std::bad_alloc&) {
    return fail(nullptr, SMLU_ERR_ALLOC, "host allocation failed");
  }
  if (rc != SMLU_OK) return fail(nullptr, rc, h->err);
  int64_t k = 0;
  auto put = [&](int64_t v) {
    if (ops && k < cap) ops[k] = v;
    ++k;
  };
  const std::vector<int>* seqs[3] = {&h->fac_comm, &h->fwd_comm, &h->bwd_comm};
  for (int q = 0; q < 3; ++q)
    for (int id : *seqs[q]) {
      const CommOp& op = h->comm[id];
      put(q);
      put(op.type);
      put(op.type == 1 ? op.root : -1);
      put(op.type == 1 ? op.bytes : 0);
      if (op.type == 1) {
        put((int64_t)op.grp.size());
        for (int32_t g : op.grp) put(g);
      } else {
        put((int64_t)op.peer.size());
        for (size_t i = 0; i < op.peer.size(); ++i) {
          put(op.peer[i]);
          put(op.sbytes[i]);
          put(op.rbytes[i]);
        }
      }
    }
  *len = k;
  if (bytes)
    for (int i = 0; i < 5; ++i) bytes[i] = h->host_bytes[i];
  if (counts) {
    counts[0] = (int64_t)h->fac.size();
    int64_t sh = 0;
    for (int64_t s = 0; s < h->plan.nsup && nparts > 1; ++s)
      if (h->plan.dist(s) && std::binary_search(h->plan.group[s].begin(), h->plan.group[s].end(), rank)) ++sh;
    counts[1] = sh;
    counts[2] = (int64_t)h->lay.blocks.size();
  }
  if (ops && k > cap) return fail(nullptr, SMLU_ERR_ARG, "ops buffer too small");
  return SMLU_OK;
}
