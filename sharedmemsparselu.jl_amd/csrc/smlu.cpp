// smlu.cpp — C-ABI of libsmlu.so (include/smlu.h): handle lifetime, the static launch
// schedule of the multifrontal refactorization and solves, device memory, factor export.
//
// Reference surface (SharedMemSparseLU.jl, src/SharedMemSparseLU.jl):
//   ParallelSparseLU(A, chunk_size)  :64-98   -> smlu_create
//   lu!(F, A)                        :245-279 -> smlu_refactor / smlu_refactor_csc
//   ldiv!(x, F, b)                   :286-342 -> smlu_solve
//   lsolve!(F, x) / rsolve!(F, x)    :349-392 -> smlu_lsolve / smlu_rsolve
//   F.L, F.U, F.p, F.q, F.Rs         :45-52   -> smlu_get_factors
//   cleanup_ParallelSparseLU!        :31      -> smlu_destroy
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <map>
#include <memory>
#include <unordered_map>
#include <string>
#include <vector>

#include "../../include/smlu.h"
#include "device.hpp"
#include "plan.hpp"

namespace smlu {
hipError_t launch_rowscale(hipStream_t, int64_t, const int64_t*, const int32_t*, const double*, double*);
hipError_t launch_fill(hipStream_t, int64_t, double*, double);
hipError_t launch_factor_reset(hipStream_t, int64_t, int32_t*, double*, int64_t, int32_t*, const int32_t*);
hipError_t launch_assemble(hipStream_t, int64_t, const XCol*, const XContrib*, const int2*, const SNode*,
                           const int32_t*, const double*, const int32_t*, const double*, double*, double*);
hipError_t launch_front_small(hipStream_t, int, int, const int32_t*, const SNode*, const int32_t*, const int32_t*,
                              const int2*, const double*, const int32_t*, const double*, double*, double*,
                            int32_t*, int32_t*, double*, double, double);
hipError_t init_kernel_attributes();
hipError_t launch_panel1(hipStream_t, int, int, int, int, int, const int32_t*, const SNode*, double*, double*,
                         int32_t*, int32_t*, int64_t, int32_t*, double*, double, int, double*, int);
hipError_t launch_step_trsm(hipStream_t, int, const FrontTile*, int, int64_t, const FrontTile*, int, int64_t,
                            int, int, const SNode*, double*, double*, int32_t*, double*, double);
hipError_t launch_laswp(hipStream_t, int64_t, const SwapTask*, int, const SNode*, double*, double*, const int32_t*,
                        int64_t);
hipError_t launch_trsm_u(hipStream_t, int64_t, const FrontTile*, int, int, int, const SNode*, double*,
                         double*, const int32_t*, int64_t);
hipError_t launch_gemm(hipStream_t, int64_t, const GemmTask*, int, int, int64_t);
hipError_t launch_gemm_g(hipStream_t, int64_t, const GemmTask*, int, int, int64_t, int32_t*, double*, double);
hipError_t launch_tri_inv(hipStream_t, int, int, const int32_t*, const SNode*, double*, double*, double*);
hipError_t launch_urows(hipStream_t, int, const URowTask*, const SNode*, double*, const double*);
hipError_t launch_fwd_tiny(hipStream_t, int, const int32_t*, const SNode*, const int32_t*, const int32_t*,
                           const int32_t*, const double*, double*, double*, Rhs, int);
hipError_t launch_bwd_tiny(hipStream_t, int, const int32_t*, const SNode*, const int32_t*, const double*, double*,
                           double*, Rhs, int);
hipError_t launch_fwd_pull(hipStream_t, int64_t, const FrontTile*, int, const SNode*, const int32_t*,
                           const int32_t*, const int32_t*, const double*, double*, Rhs);
hipError_t launch_fwd_gather(hipStream_t, int, const int32_t*, const SNode*, const int32_t*, const int32_t*,
                             const int32_t*, double*, double*, Rhs);
hipError_t launch_tri_block(hipStream_t, bool, int64_t, const FrontTile*, int, int, const SNode*,
                            const double*, double*, double*, Rhs);
hipError_t launch_bwd_u12(hipStream_t, int64_t, const FrontTile*, int, const SNode*, const int32_t*,
                          const double*, const double*, double*, Rhs);
hipError_t launch_tri_sweep(hipStream_t, bool, int64_t, const FrontTile*, int, unsigned long long*, int32_t*, double*,
                            int32_t*, const SNode*, const double*, double*, double*, Rhs, int);
hipError_t launch_fwd(hipStream_t, int, const int32_t*, const SNode*, const int32_t*, const int32_t*,
                      const int32_t*, const double*, double*, double*, Rhs);
hipError_t launch_bwd(hipStream_t, int, const int32_t*, const SNode*, const int32_t*, const double*,
                      double*, double*, Rhs);
hipError_t launch_residual(hipStream_t, int64_t, const int64_t*, const int32_t*, const int32_t*,
                           const double*, const double*, const double*, double*, double*);
hipError_t launch_axpy1(hipStream_t, int64_t, const double*, double*);
hipError_t launch_dominance(hipStream_t, int64_t, const int64_t*, const int32_t*, const int64_t*, const int32_t*,
                            const int32_t*, const double*, int32_t*);
hipError_t launch_status(hipStream_t, const int32_t*, int64_t, const SNode*, const int32_t*, int, long long*, long long);
hipError_t launch_front_hash(hipStream_t, int64_t, const SNode*, const double*, const int32_t*, unsigned long long*);
hipError_t launch_expand_z(hipStream_t, int64_t, const double*, const int64_t*, const int32_t*, double*);
hipError_t launch_perm_in(hipStream_t, int64_t, const int64_t*, const double*, const double*, double*, int,
                          int64_t, int64_t);
hipError_t launch_perm_out(hipStream_t, int64_t, const int64_t*, const double*, double*, int, int64_t, int64_t);
hipError_t launch_chunked_solve(hipStream_t, bool, int64_t, const ChunkDesc*, const double*, double*);
hipError_t launch_segcopy(hipStream_t, const SegDesc*, int64_t);
hipError_t launch_bwd_u12_cols(hipStream_t, const SNode*, int, int64_t, int64_t, int64_t, int, const int32_t*,
                               const double*, const double*, double*);
hipError_t launch_vcopy(hipStream_t, const SNode*, int, int64_t, const double*, double*);
hipError_t launch_unswap(hipStream_t, int64_t, const int64_t*, const int32_t*, const double*, double*);
}  // namespace smlu

using namespace smlu;

namespace {

constexpr int kSmallM = 128;     // fronts up to this order are factored whole in LDS
constexpr int kFullPivNs = 512;  // blocked fronts up to this many pivots search all fully-summed rows
constexpr int kNbFull = 32;
constexpr int kNbTile = 64;
constexpr int kSwapStride = 1 + 2 * 64;
constexpr int kOBDefault = 384;   // outer block of the two-level blocked front factorization (256/384/512 within 1 %; 384 best)

thread_local std::string g_last_error;

enum Kind : int {
  K_MEMSET_STORE, K_MEMSET_SCRATCH, K_SCATTER, K_EXTADD, K_FRONT_LDS, K_PANEL, K_TRSMU, K_TRSML,
  K_GEMM, K_FWD, K_BWD, K_FWDG, K_TRIF, K_BWDU, K_TRIB, K_GEMM22, K_LASWP, K_STEPTRSM, K_GEMMU,
  K_GEMMO, K_TRIINV, K_BWDU12C, K_VCOPY, K_FWDT, K_BWDT, K_SWEEPF, K_SWEEPB, K_UROWS, K_FWDP, K_NKIND
};
const char* kKindName[] = {"memset", "memset", "assemble", "assemble", "small", "panel",
                                  "trsm", "trsm", "gemm", "solve", "solve", "solve", "solve",
                                  "solve", "solve", "gemm22", "trsm", "trsm", "gemmu", "gemmo", "trsm", "solve", "solve",
                                  "solve", "solve", "solve", "solve", "urows", "solve"};
static_assert(sizeof(kKindName) / sizeof(kKindName[0]) == K_NKIND, "one kKindName entry per launch kind");
constexpr int kSolveBigNs = 256;  // fronts with more pivots use the multi-workgroup solve
// ... and so do fronts whose L panel (M x ns entries) exceeds this: one workgroup streams a
// tall panel at single-CU bandwidth (a 10^4-row front with 200 pivots took ~350 us per sweep)
constexpr int64_t kSolveBigWork = 1 << 16;
constexpr int kSolveMicroM = 8;    // tiny fronts with M <= 8: eight per wave (k_fwd_micro / k_bwd_micro)
constexpr int kSolveTinyM = 128;   // fronts with M <= 128 rows and ns <= 64: one wave each (k_fwd_tiny / k_bwd_tiny)

struct Launch {
  int kind = 0;
  int node = 0;                           // K_BWDU12C / K_VCOPY: front or block node
  int step = 0;
  int64_t off = 0, cnt = 0, nwg = 0, aux = 0, aux2 = 0;
  int64_t off2 = 0, cnt2 = 0, nwg2 = 0;   // second work list (merged launches)
  double flops = 0;
};

template <class T>
struct DBuf {
  T* p = nullptr;
  size_t n = 0;
  hipError_t alloc(size_t cnt) {
    n = cnt;
    if (cnt == 0) return hipSuccess;
    return hipMalloc((void**)&p, cnt * sizeof(T));
  }
  hipError_t upload(const T* h, size_t cnt, hipStream_t st) {
    hipError_t e = alloc(cnt);
    if (e != hipSuccess || cnt == 0) return e;
    return hipMemcpyAsync(p, h, cnt * sizeof(T), hipMemcpyHostToDevice, st);
  }
  void free() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
};

// Host description of one copy of a pack / unpack step, resolved to device addresses once the
// buffers exist: base 0 store, 1 scratch, 2 vbuf, 3 wrk (x), 4 send staging, 5 receive staging,
// 6 broadcast block buffer, 7 tile inverses, 8 swap lists, 9 rowperm; offsets in bytes.
struct HSeg {
  int sb;
  int64_t so;
  int db;
  int64_t dof;
  int64_t bytes;
};

// One communication step between segments of the schedule.
struct CommOp {
  int type = 0;                          // 0: exchange with peers, 1: broadcast within a group
  std::vector<int32_t> peer;             // exchange: peers (ascending)
  std::vector<int> sbase, rbase;         // per peer: buffer (HSeg base ids) and byte offsets
  std::vector<int64_t> soff, roff, sbytes, rbytes;
  int32_t root = -1;                     // broadcast: root and group (ascending, includes root)
  std::vector<int32_t> grp;
  int bbase = 4;                         // broadcast buffer: send staging on the root, the
  int64_t bytes = 0;                     //   block buffer elsewhere
  std::vector<HSeg> pack, unpack;        // copies before / after the transfer
  int64_t pack0 = 0, unpack0 = 0;        // ranges in the device descriptor array
  // per-peer helpers used while the schedule is built
  int at(int32_t p) {
    for (size_t i = 0; i < peer.size(); ++i)
      if (peer[i] == p) return (int)i;
    peer.push_back(p);
    sbase.push_back(4);
    rbase.push_back(5);
    soff.push_back(0);
    roff.push_back(0);
    sbytes.push_back(0);
    rbytes.push_back(0);
    return (int)peer.size() - 1;
  }
};

// ---- built-in RCCL transport (librccl loaded at run time: the library itself needs RCCL only
// when a caller asks for it) ------------------------------------------------------------------
struct RcclApi {
  void* lib = nullptr;
  ncclResult_t (*GetUniqueId)(ncclUniqueId*);
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int);
  ncclResult_t (*CommDestroy)(ncclComm_t);
  ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t);
  ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t);
  ncclResult_t (*GroupStart)();
  ncclResult_t (*GroupEnd)();
  ncclResult_t (*AllReduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t);
  ncclResult_t (*CommCount)(const ncclComm_t, int*);
};

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

struct RcclState {
  ncclComm_t comm = nullptr;
  int rank = 0;
  int comm_count = 0;             // ranks in the communicator (ncclCommCount after init)
  hipStream_t stream = nullptr;   // the handle's stream (allreduce)
  double* dbuf = nullptr;         // device scratch for the allreduce
};

// point-to-point batch over xGMI: sends and receives of all peers in one group
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

}  // namespace

struct smlu_plan {
  Plan plan;
};

struct smlu_handle {
  smlu_opts opts{};
  Plan plan;
  int device = 0;
  hipStream_t stream = nullptr;
  std::string err;
  int64_t errcol = -1;
  bool have_numeric = false;
  bool given_Rs = false;
  // device buffers
  DBuf<double> A, Rs, store, scratch, wrk, wrk2, vbuf, growth;
  DBuf<double> vbufm, wrkm, wrk2m;   // multi-RHS solve: kMultiRhs copies of vbuf / wrk / wrk2 (on first use)
  DBuf<double> tinv;   // per (front, sub-panel) slot: I - L_kk^-1 and I - U_kk^-1 (GEMM-form TRSM)
  // the reference's dense-chunk solve layout, rebuilt after each factorization
  DBuf<double> ch_data;
  DBuf<ChunkDesc> ch_desc;   // L chunks [0, ch_T), U chunks [ch_T, 2 ch_T)
  DBuf<int64_t> ch_p, ch_q;
  int64_t ch_T = 0, ch_size = 0, ch_version = -1;
  int64_t nfactor = 0;       // completed numeric factorizations
  DBuf<double> ref_b, ref_r, ref_d, ref_nrm;   // iterative refinement (allocated on first use)
  DBuf<int32_t> Acol;                          // column of each A entry (residuals, dominance check)
  DBuf<int64_t> Acolp;                         // A's colptr (device dominance check)
  DBuf<int32_t> domflag;
  int refine_steps = 0;
  double refine_berr = -1;   // componentwise backward error at the last refinement check
  double refine_resid = -1;
  DBuf<int64_t> Arowptr, p0, q, posfirst;
  DBuf<int32_t> Arow_ent, Arow, rows, relmap, chlist, ilist, rowperm, rowperm0, info, swaps;
  DBuf<SNode> sn;
  DBuf<XContrib> xtasks;
  DBuf<int2> aents;
  DBuf<FrontTile> ftiles;
  DBuf<int32_t> gptr, gent;       // pull lists of the large fronts' forward gather (k_fwd_pull)
  DBuf<int32_t> ssync, sstatus;   // sync-free solve sweeps: block flags (epochs, never reset); timeouts
  DBuf<unsigned long long> stick; // ... one monotone ticket counter per sweep launch
  DBuf<double> sxh;               // ... hand-off slots: 64 x kMultiRhs doubles per flag
  int64_t ssync_n = 0;
  DBuf<GemmTask> gtasks;
  DBuf<SwapTask> stasks;
  DBuf<URowTask> urtasks;     // fused U-row tasks (k_urows)
  DBuf<XCol> xcols;
  // schedule
  std::vector<Launch> fac, fwd, bwd;
  std::vector<Launch> fwdm, bwdm;   // per-block launches instead of sweeps: batched right-hand sides (one
                                    // GPU) and the re-run of a solve whose sweep wait timed out
  std::vector<size_t> fwdm_seg, bwdm_seg;   // their segment starts (the comm steps of fwd / bwd)
  std::vector<SNode> hsn;
  double gemm_flops = 0, gemm22_flops = 0, dense_flops = 0;
  int64_t gemm_launches = 0, gemm128_launches = 0;
  double gemm_bytes = 0;      // algorithmic bytes of the GEMM launches: A, B read, C read + written
  int64_t nlaunch = 0;
  // stats
  double refactor_ms = 0, solve_ms = 0, growth_max = 0;
  int64_t weak = 0;
  double kind_ms[K_NKIND] = {0};
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_pool;
  std::vector<int> ev_kind;
  hipStream_t caller = nullptr;   // caller's stream (smlu_set_stream; nullptr = the null stream)
  hipEvent_t ev_caller = nullptr;
  DBuf<long long> rb;         // status record for the host (k_status; read_status)
  // the caller's L/U pattern (smlu_create_with_pivots, UMFPACK's F.L / F.U): when present, the
  // factors are exported on exactly that pattern; pattern_dropped counts the structural entries of
  // (Rs.*A)[p, q]'s fill it leaves out (UMFPACK drops entries that are exactly zero)
  std::vector<int64_t> gLp, gLi, gUp, gUi;
  bool given_pattern = false;
  int64_t pattern_dropped = 0;
  long long rb_seq = 0;       // sequence number of the last status record
  int64_t status_copy_retries = 0;   // status records re-read after a stamp mismatch
  int64_t bad_info_node = -1, bad_info_count = 0;   // illegal info words seen by k_status
  int32_t bad_info_word = 0;
  int64_t sweep_timeouts = 0;   // solves re-run on the per-block schedule after a sweep wait timed out
  int sweep_spin = 1 << 22;     // polls before a sweep wait gives up (SMLU_SWEEP_SPIN; 0 = always, tests)
  DBuf<double> bstash;          // the solve's input when the final step overwrites it (x === b, lsolve!/rsolve!)
  std::vector<std::pair<int, hipGraphExec_t>> sol_execs;   // captured solve sweeps, keyed by mode/rhs count
  std::vector<hipGraphExec_t> fac_execs;   // one captured graph per factor segment
  int fac_exec_profile = -1;
  std::vector<std::pair<size_t, size_t>> seg_events;   // profile events of each captured segment
  // multi-GPU partition (smlu_dist_*): this rank's fronts and column blocks (RankLayout), the
  // schedule cut into segments at the communication steps
  int rank = 0, nranks = 1;
  RankLayout lay;
  int64_t nnodes = 0;                              // fronts + block nodes of shared fronts
  std::vector<int32_t> node_front;                 // node -> front
  std::vector<size_t> fac_seg, fwd_seg, bwd_seg;   // launch index where each segment starts
  std::vector<int> fac_comm, fwd_comm, bwd_comm;   // comm op run before segment k >= 1
  std::vector<CommOp> comm;
  smlu_transport tr{};
  void* rccl = nullptr;                            // built-in RCCL transport state
  DBuf<double> stage_s, stage_r, bcbuf, d_red;
  DBuf<SegDesc> segdesc;
  char* hstage_s = nullptr;                        // pinned host staging (host-memory transports)
  char* hstage_r = nullptr;
  int64_t stage_bytes_s = 0, stage_bytes_r = 0;
  // bytes this rank sent / received through the transport (cumulative, and in the last refactor)
  double comm_sent = 0, comm_recv = 0, comm_sent_fac = 0, comm_recv_fac = 0;
  int64_t comm_calls = 0;
  size_t fac_graph_events = 0;
  bool graph_failed = false;
  int ob = kOBDefault;        // outer block width (SMLU_OB overrides; multiple of 64)
  int64_t t128_min = 512;     // 128x128 GEMM tiles when a launch has at least this many
  bool small_k = true;        // k <= 64 launches use k_gemm_k64 (SMLU_SMALLK=0: off)
  bool dominant = false;      // A diagonally dominant (by rows or columns): last host values seen
  int pivmode = 0;            // 0: diagonal-tile pivoting for large (and, if dominant, mid-size)
                              //    fronts; 1: full-candidate pivoting in every blocked front (the
                              //    re-pivoting refactor after a zero or weak tile pivot)
  int64_t repivots = 0;       // re-pivoting refactors run so far
  int64_t flag_node = -1;     // first flagged node of the last factorization and its info word
  int32_t flag_info = 0;
  int64_t repivot_node = -1;  // what triggered the last re-pivot: the first flagged node, its info
  int32_t repivot_info = 0;   //   word (bit 0 zero pivot, bit 1 weak pivot) and the growth seen
  double repivot_growth = 0;
  SNode repivot_sn{};         //   and that node's record (mode, ns, nu) in the schedule that flagged it
  bool trsm_gemm = true;      // GEMM-form triangular solves of the blocked fronts
  // ComplexF64 handle (smlu_create_z): the plan and factors are those of the real-equivalent K
  bool zc = false;
  bool cpair = false;                // pair-preserving pivots (complex handle, no row transversal)
  int64_t zn = 0, znnz = 0;          // complex n and nnz(A)
  std::vector<int64_t> zdst;         // per complex entry: K position of its (re, im) in column 2j
  std::vector<int32_t> zoff;         // ... and the distance to its (-im, re) in column 2j+1
  std::vector<int64_t> zcolptr, zrowval;   // complex pattern (0-based), for pattern checks
  DBuf<int64_t> d_zdst;
  DBuf<int32_t> d_zoff;
  ~smlu_handle() { release_all(); }
  void release_buffers() {
    if (stream) (void)hipSetDevice(device);
    release_graphs();
    DBuf<double>* d[] = {&A, &Rs, &store, &scratch, &wrk, &wrk2, &vbuf, &vbufm, &wrkm, &wrk2m, &growth, &ref_b, &ref_r, &ref_d, &ref_nrm,
                         &tinv, &ch_data, &bstash};
    ch_desc.free();
    ch_p.free();
    ch_q.free();
    ch_version = -1;
    Acol.free();
    Acolp.free();
    domflag.free();
    for (auto* b : d) b->free();
    DBuf<int64_t>* l[] = {&Arowptr, &p0, &q, &posfirst};
    for (auto* b : l) b->free();
    DBuf<int32_t>* i[] = {&Arow_ent, &Arow, &rows, &relmap, &chlist, &ilist, &rowperm, &rowperm0, &info, &swaps};
    for (auto* b : i) b->free();
    sn.free();
    d_zdst.free();
    d_zoff.free();
    xtasks.free();
    aents.free();
    ftiles.free();
    gptr.free();
    gent.free();
    ssync.free();
    sstatus.free();
    stick.free();
    sxh.free();
    gtasks.free();
    stasks.free();
    urtasks.free();
    xcols.free();
    stage_s.free();
    stage_r.free();
    bcbuf.free();
    segdesc.free();
    d_red.free();
    if (hstage_s) (void)hipHostFree(hstage_s);
    if (hstage_r) (void)hipHostFree(hstage_r);
    hstage_s = hstage_r = nullptr;
  }
  void release_graphs() {
    for (auto& g : fac_execs)
      if (g) (void)hipGraphExecDestroy(g);
    fac_execs.clear();
    for (auto& g : sol_execs)
      if (g.second) (void)hipGraphExecDestroy(g.second);
    sol_execs.clear();
    fac_exec_profile = -1;
  }
  void release_all() {
    release_graphs();
    release_buffers();
    if (rccl) {
      if (RcclApi* R = rccl_api()) (void)R->CommDestroy(static_cast<RcclState*>(rccl)->comm);
      delete static_cast<RcclState*>(rccl);
      rccl = nullptr;
    }
    for (auto& e : ev_pool) {
      (void)hipEventDestroy(e.first);
      (void)hipEventDestroy(e.second);
    }
    ev_pool.clear();
    ev_kind.clear();
    rb.free();
    if (ev_caller) (void)hipEventDestroy(ev_caller);
    if (stream) (void)hipStreamDestroy(stream);
    stream = nullptr;
  }
};

#define HIPCHK2(hh, expr)                                                            \
  do {                                                                               \
    hipError_t _e = (expr);                                                          \
    if (_e != hipSuccess) {                                                          \
      (hh)->err = std::string("HIP error: ") + hipGetErrorString(_e) + " at " #expr; \
      g_last_error = (hh)->err;                                                      \
      return SMLU_ERR_HIP;                                                           \
    }                                                                                \
  } while (0)

#define HIPCHK(expr)                                                                 \
  do {                                                                               \
    hipError_t _e = (expr);                                                          \
    if (_e != hipSuccess) {                                                          \
      h->err = std::string("HIP error: ") + hipGetErrorString(_e) + " at " #expr;    \
      g_last_error = h->err;                                                         \
      return SMLU_ERR_HIP;                                                           \
    }                                                                                \
  } while (0)

static int fail(smlu_handle* h, int code, const std::string& msg) {
  if (h) h->err = msg;
  g_last_error = msg;
  return code;
}

static PlanOptions plan_opts(const smlu_opts& o) {
  PlanOptions p;
  p.ordering = o.ordering;
  for (int i = 0; i < 3; ++i) p.grid[i] = o.grid[i];
  p.relax = o.relax;
  p.leaf_size = o.leaf_size > 0 ? o.leaf_size : 64;
  return p;
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

// ---------------------------------------------------------------------------------------
// Schedule construction (host, once per plan)
// ---------------------------------------------------------------------------------------
static int build_schedule(smlu_handle* h) {
  Plan& P = h->plan;
  const Tune tn = tune();
  const int64_t nsup = P.nsup;
  hipStream_t st = h->stream;
  // supernode records: fronts [0, nsup) with this rank's offsets (RankLayout); a shared front
  // (multi-GPU) keeps a front node for its solves and the row maps, plus one block node per
  // owned column block whose offsets are shifted so that the front's column c of the block sits
  // at the usual place (pivot block: L + c*M; update block: U + (c-ns)*ns, F + (c-ns)*nu)
  const RankLayout& Y = h->lay;
  h->hsn.resize(nsup);
  int64_t voff = 0;
  // Largest ns factored with full-candidate pivoting.  A diagonally dominant matrix needs no
  // row exchanges (partial pivoting keeps the diagonal and the Schur complements stay
  // dominant), so there the mid-size fronts take the faster diagonal-tile path too; its growth
  // check still flags weak pivots if a refactor's new values lose dominance (refinement then
  // runs in the solves).  SMLU_FULLPIV_NS overrides (dev).
  // a complex handle's pair-preserving pivots search every fully-summed row (mode 1): the
  // diagonal-tile panels have no pair rule
  const int64_t full_piv_ns = (h->pivmode == 1 || h->cpair) ? std::numeric_limits<int64_t>::max()
                              : tn.fullpiv_ns >= 0 ? tn.fullpiv_ns
                              : h->dominant ? (int64_t)kSmallM : (int64_t)kFullPivNs;
  for (int64_t s = 0; s < nsup; ++s) {
    SNode r{};
    r.first = P.s_first[s];
    r.Loff = Y.Loff[s] >= 0 ? Y.Loff[s] : 0;
    r.Uoff = Y.Uoff[s] >= 0 ? Y.Uoff[s] : 0;
    r.Foff = Y.Foff[s];
    r.rowptr = P.s_rowptr[s];
    r.voff = voff;
    r.ns = (int32_t)P.ns(s);
    r.nu = (int32_t)P.nu(s);
    voff += P.M(s);
    r.parent = (int32_t)P.s_parent[s];
    int64_t M = P.M(s);
    if (M <= kSmallM) { r.mode = 0; r.nb = 0; }
    else if (r.ns <= full_piv_ns) { r.mode = 1; r.nb = kNbFull; }
    else { r.mode = 2; r.nb = kNbTile; }
    if (h->opts.pivot_tol <= 0) { /* no pivoting requested: tile mode never searches far */ }
    r.chbeg = (int32_t)P.ch_ptr[s];
    r.chend = (int32_t)P.ch_ptr[s + 1];
    r.level = P.s_level[s];
    r.cpair = h->cpair ? 1 : 0;
    if (h->nranks > 1 && P.dist(s)) { r.mode = 2; r.nb = kNbTile; }   // shared fronts: diagonal-tile pivoting
    h->hsn[s] = r;
  }
  h->node_front.resize(nsup);
  for (int64_t s = 0; s < nsup; ++s) h->node_front[s] = (int32_t)s;
  std::vector<int32_t> blknode(Y.blocks.size());
  std::unordered_map<int64_t, int32_t> blkmap;   // (front, block) -> index in Y.blocks
  for (size_t i = 0; i < Y.blocks.size(); ++i) {
    const RankLayout::Blk& B = Y.blocks[i];
    SNode r = h->hsn[B.s];
    const int64_t ns = r.ns, nu = r.nu, M = ns + nu;
    if (B.c0 < ns) {
      r.Loff = B.loff - B.c0 * M;
    } else {
      r.Uoff = B.loff - (B.c0 - ns) * ns;
      r.Foff = B.foff - (B.c0 - ns) * nu;
    }
    blknode[i] = (int32_t)h->hsn.size();
    blkmap[(int64_t)B.s * 1048576 + B.b] = (int32_t)i;
    h->hsn.push_back(r);
    h->node_front.push_back(B.s);
  }
  h->nnodes = (int64_t)h->hsn.size();
  // given (p,q): no pivoting on top of the caller's order -> tile mode pivots only if the
  // diagonal is exactly zero; we force diag preference by a tiny diag tolerance at launch.
  std::vector<int32_t> ilist;
  std::vector<XContrib> xt;
  std::vector<FrontTile> ft;
  std::vector<int32_t> gptr, gent;   // k_fwd_pull lists
  std::vector<GemmTask> gt;
  std::vector<SwapTask> st_tasks;
  std::vector<URowTask> ur_tasks;
  std::vector<XCol> xc;
  std::vector<int2> ae;
  // A entries grouped by front, sorted by (local column, local row)
  std::vector<int64_t> fr_ptr(nsup + 1, 0);
  std::vector<int32_t> fr_ent((size_t)P.nnzA);
  {
    for (int64_t e = 0; e < P.nnzA; ++e) ++fr_ptr[P.A_s[e] + 1];
    for (int64_t s = 0; s < nsup; ++s) fr_ptr[s + 1] += fr_ptr[s];
    std::vector<int64_t> fp(fr_ptr.begin(), fr_ptr.end() - 1);
    for (int64_t e = 0; e < P.nnzA; ++e) fr_ent[fp[P.A_s[e]]++] = (int32_t)e;
    for (int64_t s = 0; s < nsup; ++s)
      std::sort(fr_ent.begin() + fr_ptr[s], fr_ent.begin() + fr_ptr[s + 1], [&](int32_t a, int32_t b) {
        return P.A_lj[a] != P.A_lj[b] ? P.A_lj[a] < P.A_lj[b] : P.A_li[a] < P.A_li[b];
      });
  }
  double* store = h->store.p;
  double* scratch = h->scratch.p;
  h->fac.clear();
  // this rank's fronts by level (every front when nranks == 1)
  std::vector<int64_t> LP(P.nlevels + 1, 0);
  std::vector<int32_t> LS;
  std::vector<std::vector<int32_t>> dfront(P.nlevels);   // shared fronts this rank works on, per level
  std::vector<char> dlevel(P.nlevels, 0);          // a level holding any shared front (any rank)
  for (int l = 0; l < P.nlevels; ++l) {
    for (int64_t k = P.lev_ptr[l]; k < P.lev_ptr[l + 1]; ++k) {
      const int64_t s = P.lev_sup[k];
      if (h->nranks == 1) { LS.push_back((int32_t)s); continue; }
      if (!P.dist(s)) {
        if (P.owner[s] == h->rank) LS.push_back((int32_t)s);
        continue;
      }
      dlevel[l] = 1;
      if (std::binary_search(P.group[s].begin(), P.group[s].end(), h->rank)) dfront[l].push_back((int32_t)s);
    }
    LP[l + 1] = (int64_t)LS.size();
  }
  h->fac_seg.assign(1, 0);
  h->fwd_seg.assign(1, 0);
  h->bwd_seg.assign(1, 0);
  h->fac_comm.clear();
  h->fwd_comm.clear();
  h->bwd_comm.clear();
  h->comm.clear();
  // a communication step ends the current segment of `seq`
  auto add_comm = [&](std::vector<Launch>& seq, std::vector<size_t>& seg, std::vector<int>& cm, CommOp&& op) {
    seg.push_back(seq.size());
    cm.push_back((int)h->comm.size());
    h->comm.push_back(std::move(op));
  };
  const int dist_slots = h->nranks > 1 ? h->ob / 32 : 0;   // swap / tile-inverse slots of the shared front
  // where child column jc of c lives: (rank, scratch offset on that rank if it is this rank)
  auto child_col = [&](int64_t c, int64_t jc, int64_t* src) -> int32_t {
    const int64_t nuc = P.nu(c);
    if (!P.dist(c)) {
      if (src && P.owner[c] == h->rank) *src = Y.Foff[c] + jc * nuc;
      return P.owner[c];
    }
    const int64_t b = P.npblk(c) + jc / P.dob;
    const int32_t o = P.blk_owner(c, b);
    if (src && o == h->rank) {
      const RankLayout::Blk& B = Y.blocks[blkmap.at((int64_t)c * 1048576 + b)];
      *src = B.foff + (P.ns(c) + jc - B.c0) * nuc;
    }
    return o;
  };
  if (tn.ob > 0) h->ob = tn.ob;
  h->t128_min = tn.t128_min;
  h->small_k = tn.small_k;
  // MFMA 128 tile: code 131 (v3: LDS-DMA staging, kernels_gemm.hip); the F22 launches (k = ns, the
  // long-k shapes) take 135, the same tile with the next slice's barrier between its last two
  // k-quads (+3 % at k >= 2048, neutral at the k = 384 trailing shapes: tools/gemm_bench)
  const int mfma_tile = 131;
  // GEMM-form TRSM (k_tri_inv + GEMM tasks) needs the growth epilogue of the MFMA/64 tiles
  // (the 32-wide panels keep k_step_trsm: measured best)
  h->trsm_gemm = h->opts.use_mfma;
  // GEMM tasks whose A or B operand lives in the tinv buffer (allocated after the schedule)
  std::vector<std::pair<int64_t, int64_t>> tinv_patch;   // (gt index * 2 + operand B?, offset)
  h->gemm_flops = 0;
  h->gemm_launches = h->gemm128_launches = 0;
  h->gemm_bytes = 0;
  h->gemm22_flops = 0;
  h->dense_flops = P.flops;
  int64_t max_list = 1;
  // GEMM launches: 128x128 tiles when the launch has enough of them to fill the GPU,
  // otherwise 64x64 tiles (same per-element arithmetic, bitwise-identical results).
  auto add_gemm_launch = [&](std::vector<GemmTask>& cand, double fl, int step, int kind = K_GEMM,
                             const std::vector<int64_t>* tpatch = nullptr) {
    if (cand.empty()) return;
    const bool count = kind != K_TRSML;   // GEMM-form TRSM is accounted as "trsm", not GEMM
    int64_t t128 = 0;
    for (auto& g : cand) t128 += (int64_t)((g.m + 127) / 128) * ((g.n + 127) / 128);
    int tile = t128 >= h->t128_min ? 128 : 64;
    if (tile == 128 && h->opts.use_mfma) tile = mfma_tile;   // fp64 MFMA variant of the 128 tile
    if (tile == 131 && step < 0) tile = 135;
    if (tile == 64 && h->small_k) {                    // every k <= 64: one-shot K staging
      int kmax = 0;
      for (auto& g : cand) kmax = std::max(kmax, g.k);
      if (kmax <= 64) tile = 65;
    }
    if (step < 0 && !tpatch)   // F22: longest k first, so the launch's last tiles are short ones
      std::stable_sort(cand.begin(), cand.end(), [](const GemmTask& a, const GemmTask& b) { return a.k > b.k; });
    Launch L;
    L.kind = step < 0 ? K_GEMM22 : kind;
    L.step = step;
    L.off = (int64_t)gt.size();
    L.aux = tile;
    int64_t tiles = 0;
    const int ts = tile >= 128 ? 128 : 64;
    for (size_t i = 0; i < cand.size(); ++i) {
      GemmTask& g = cand[i];
      if (count) h->gemm_bytes += 8.0 * ((double)g.m * g.k + (double)g.k * g.n + 2.0 * g.m * g.n);
      if (tpatch && (*tpatch)[i] >= 0) tinv_patch.push_back({(int64_t)gt.size(), (*tpatch)[i]});
      g.tiles_m = (g.m + ts - 1) / ts;
      g.tile0 = tiles;
      tiles += (int64_t)g.tiles_m * ((g.n + ts - 1) / ts);
      gt.push_back(g);
    }
    L.cnt = (int64_t)cand.size();
    L.nwg = tiles;
    L.flops = fl;
    h->fac.push_back(L);
    if (!count) return;
    h->gemm_flops += fl;
    ++h->gemm_launches;
    if (tile >= 128) ++h->gemm128_launches;
    if (step < 0) h->gemm22_flops += fl;
  };
  // fronts whose triangular solves run in GEMM form (tile inverses); they also take the
  // super-block level of the three-level blocking (SB columns; OB for the others)
  auto gform = [&](int64_t s) {
    return h->trsm_gemm && h->hsn[s].nb == kNbTile;
  };
  const int64_t spf = h->ob / 32;   // swap / tile-inverse slots per front
  // fused panels (k_panel_blk<16, true>: panel + tile inverses + in-block row interchanges) for
  // the GEMM-form fronts (every 64-wide panel then belongs to one); SMLU_FUSED_PANEL=0: three launches
  // 2 (default): panel + the in-block row interchanges (no k_laswp inside the block) + the tile
  // inverses by 16 x 16 blocks on the matrix cores (no k_tri_inv); 1: without the inverses;
  // 0: three launches
  const int fuse_mode = !(h->trsm_gemm && h->ob <= 64 + 16 * 20) ? 0 : 2;
  const bool fuse_panel = fuse_mode > 0, fuse_inv = fuse_mode == 2;
  // fused U rows at the end of an outer block (k_urows) for the GEMM-form fronts; SMLU_FUSED_UROWS=0:
  // one TRSM + one update launch per sub-panel
  const bool fuse_urows = h->ob <= 384;
  // tinv operand encoding in tpatch: offset * 2 + (1 if the operand is B, 0 if A)
  auto tinv_slot_off = [](int64_t slot, bool upper) { return slot * 8192 + (upper ? 4096 : 0); };
  for (int l = 0; l < P.nlevels; ++l) {
    Launch L;
    // (shared fronts of this level, in front order on every rank)
    // shared front: the children's F22 columns move to the owners of the target columns; a
    // rank receives them into its receive area ordered by (source rank, child, column)
    std::unordered_map<int64_t, int64_t> recv_at;   // (child, column) -> scratch offset
    for (const int32_t t : dfront[l]) {
      CommOp op;
      std::vector<std::vector<std::pair<int64_t, int64_t>>> from(h->nranks);   // per source: (c, jc)
      for (int64_t e = P.ch_ptr[t]; e < P.ch_ptr[t + 1]; ++e) {
        const int64_t c = P.ch_list[e];
        const int32_t* rm = P.relmap.data() + P.s_rowptr[c];
        const int64_t nuc = P.nu(c);
        for (int64_t jc = 0; jc < nuc; ++jc) {
          const int32_t dst = P.col_owner(t, rm[jc]);
          int64_t src = -1;
          const int32_t o = child_col(c, jc, &src);
          if (o == dst) continue;
          if (o == h->rank) {            // send: pack into the staging buffer
            const int pi = op.at(dst);
            op.pack.push_back(HSeg{1, 8 * src, 4, 0, 8 * nuc});   // staging offset fixed below
            op.pack.back().db = 1000 + pi;                           // peer marker
            op.sbytes[pi] += 8 * nuc;
          } else if (dst == h->rank) {
            from[o].push_back({c, jc});
          }
        }
      }
      int64_t ro = Y.recv_off[t];
      for (int32_t o = 0; o < h->nranks; ++o) {
        if (from[o].empty()) continue;
        const int pi = op.at(o);
        op.rbase[pi] = 1;
        op.roff[pi] = 8 * ro;
        for (auto& cj : from[o]) {
          recv_at[cj.first * 1048576 + cj.second] = ro;
          ro += P.nu(cj.first);
          op.rbytes[pi] += 8 * P.nu(cj.first);
        }
      }
      // send staging offsets: per peer contiguous, in (child, column) order
      {
        std::vector<int64_t> base(op.peer.size(), 0);
        int64_t acc = 0;
        for (size_t i = 0; i < op.peer.size(); ++i) {
          op.soff[i] = acc;
          base[i] = acc;
          acc += op.sbytes[i];
        }
        for (auto& g : op.pack) {
          const int pi = g.db - 1000;
          g.db = 4;
          g.dof = base[pi];
          base[pi] += g.bytes;
        }
      }
      add_comm(h->fac, h->fac_seg, h->fac_comm, std::move(op));
    }
    // assembly: every column of this level's fronts built once (zeros, scaled A entries, the
    // children's F22 columns in child order) -- k_assemble, one wave per column
    {
      L = Launch();
      L.kind = K_EXTADD;
      L.off = (int64_t)xc.size();
      std::vector<int32_t> cnt, pos;
      auto front_columns = [&](int64_t s, const std::vector<std::pair<int64_t, int64_t>>& ranges,
                               const std::vector<int32_t>& nodes) {
        const int64_t M = P.M(s);
        cnt.assign(M + 1, 0);
        for (int64_t ci = P.ch_ptr[s]; ci < P.ch_ptr[s + 1]; ++ci) {
          const int64_t c = P.ch_list[ci];
          const int32_t* rm = P.relmap.data() + h->hsn[c].rowptr;
          for (int64_t jc = 0; jc < P.nu(c); ++jc) ++cnt[rm[jc] + 1];
        }
        for (int64_t tj = 0; tj < M; ++tj) cnt[tj + 1] += cnt[tj];
        const int64_t base = (int64_t)xt.size();
        xt.resize(base + cnt[M]);
        pos.assign(cnt.begin(), cnt.end() - 1);
        for (int64_t ci = P.ch_ptr[s]; ci < P.ch_ptr[s + 1]; ++ci) {
          const int64_t c = P.ch_list[ci];
          const int32_t* rm = P.relmap.data() + h->hsn[c].rowptr;
          for (int64_t jc = 0; jc < P.nu(c); ++jc) {
            int64_t src = -1;
            if (h->nranks == 1) src = h->hsn[c].Foff + jc * P.nu(c);
            else if (P.col_owner(s, rm[jc]) == h->rank) {
              if (child_col(c, jc, &src) != h->rank) src = recv_at.at(c * 1048576 + jc);
            }
            xt[base + pos[rm[jc]]++] = XContrib{(int32_t)c, 0, src};
          }
        }
        // A entries of this front by (column, row); one task per column of the given ranges
        int64_t ea = fr_ptr[s];
        const int64_t eb = fr_ptr[s + 1];
        for (size_t ri = 0; ri < ranges.size(); ++ri)
          for (int64_t tj = ranges[ri].first; tj < ranges[ri].second; ++tj) {
            while (ea < eb && P.A_lj[fr_ent[ea]] < tj) ++ea;
            const int64_t a0 = (int64_t)ae.size();
            while (ea < eb && P.A_lj[fr_ent[ea]] == tj) {
              ae.push_back(make_int2(fr_ent[ea], P.A_li[fr_ent[ea]]));
              ++ea;
            }
            xc.push_back(XCol{nodes[ri], (int32_t)tj, base + cnt[tj], cnt[tj + 1] - cnt[tj],
                              (int32_t)((int64_t)ae.size() - a0), a0});
          }
      };
      for (int64_t k = LP[l]; k < LP[l + 1]; ++k) {   // small fronts assemble inside k_front_small
        const int64_t s = LS[k];
        if (h->hsn[s].mode != 0) front_columns(s, {{0, P.M(s)}}, {(int32_t)s});
      }
      for (const int32_t t : dfront[l]) {   // the shared front: this rank's column blocks
        std::vector<std::pair<int64_t, int64_t>> ranges;
        std::vector<int32_t> nodes;
        for (size_t i = 0; i < Y.blocks.size(); ++i)
          if (Y.blocks[i].s == t) {
            ranges.push_back({Y.blocks[i].c0, Y.blocks[i].c1});
            nodes.push_back(blknode[i]);
          }
        front_columns(t, ranges, nodes);
      }
      L.cnt = (int64_t)xc.size() - L.off;
      if (L.cnt > 0) h->fac.push_back(L);
    }
    // small fronts (assembly fused into the factorization), launched per size class so that
    // small fronts get small LDS (occupancy); ilist: (front, first A entry, A entry count), the
    // front's A entries as (entry, local column << 16 | local row)
    {
      const int64_t cls[6] = {16, 32, 48, 64, 96, kSmallM};
      for (int c = 0; c < 6; ++c) {
        L = Launch();
        L.kind = K_FRONT_LDS;
        L.off = (int64_t)ilist.size();
        int64_t Mmax = 0;
        for (int64_t k = LP[l]; k < LP[l + 1]; ++k) {
          int64_t s = LS[k];
          if (h->hsn[s].mode != 0) continue;
          int64_t M = P.M(s);
          if (M > cls[c] || (c > 0 && M <= cls[c - 1])) continue;
          ilist.push_back((int32_t)s);
          ilist.push_back((int32_t)ae.size());
          ilist.push_back((int32_t)(fr_ptr[s + 1] - fr_ptr[s]));
          for (int64_t e = fr_ptr[s]; e < fr_ptr[s + 1]; ++e) {
            const int32_t id = fr_ent[e];
            ae.push_back(make_int2(id, (int32_t)((P.A_lj[id] << 16) | P.A_li[id])));
          }
          Mmax = std::max(Mmax, M);
        }
        L.cnt = ((int64_t)ilist.size() - L.off) / 3;
        L.aux = Mmax;
        if (L.cnt > 0) h->fac.push_back(L);
      }
    }
    // blocked fronts
    std::vector<int64_t> big;
    std::unordered_map<int64_t, int64_t> bidx;   // front -> index in big (swap-list slots)
    int64_t maxsteps = 0;
    for (int64_t k = LP[l]; k < LP[l + 1]; ++k) {
      int64_t s = LS[k];
      const SNode& r = h->hsn[s];
      if (r.mode == 0) continue;
      bidx[s] = (int64_t)big.size();
      big.push_back(s);
      maxsteps = std::max<int64_t>(maxsteps, (r.ns + r.nb - 1) / r.nb);
    }
    max_list = std::max<int64_t>(max_list, dist_slots + (int64_t)big.size() * spf);
    // swap-list slot of sub-panel u of a front's current outer block
    auto slot_of = [&](int64_t s, int64_t u) { return dist_slots + bidx[s] * spf + u; };
    for (int64_t t = 0; t < maxsteps; ++t) {
      std::vector<int64_t> act;
      for (auto s : big) {
        const SNode& r = h->hsn[s];
        if (t * r.nb < r.ns) act.push_back(s);
      }
      if (act.empty()) continue;
      // panel launch classes by register-kernel shape: (W=64, 1 wave), (W=32, 1/2/4/8 waves)
      auto pclass = [&](int64_t s) {
        const SNode& r = h->hsn[s];
        int64_t kb = t * r.nb, w = std::min<int64_t>(r.nb, r.ns - kb);
        int64_t R = r.mode == 1 ? r.ns - kb : w;
        if (r.nb > 32) return 0;
        return R <= 64 ? 1 : R <= 128 ? 2 : R <= 256 ? 3 : R <= 512 ? 4 : 5;
      };
      std::stable_sort(act.begin(), act.end(), [&](int64_t a, int64_t b) { return pclass(a) < pclass(b); });
      {
        size_t pos = 0;
        for (int c = 0; c < 6 && pos < act.size(); ++c) {
          L = Launch();
          L.kind = K_PANEL;
          L.step = (int)t;
          L.off = (int64_t)ilist.size();
          int64_t rmax = 1, wmax = 1, cnt = 0;
          while (pos < act.size() && pclass(act[pos]) == c) {
            const SNode& r = h->hsn[act[pos]];
            int64_t kb = t * r.nb, w = std::min<int64_t>(r.nb, r.ns - kb);
            rmax = std::max(rmax, r.mode == 1 ? r.ns - kb : w);
            wmax = std::max<int64_t>(wmax, r.nb);
            ilist.push_back((int32_t)act[pos]);
            ilist.push_back((int32_t)slot_of(act[pos], t % (h->ob / r.nb)));
            ++pos;
            ++cnt;
          }
          L.cnt = cnt;
          L.aux = 0;
          L.nwg = rmax;
          L.aux2 = wmax;
          L.cnt2 = c == 0 ? fuse_mode : 0;   // 64-wide panels of GEMM-form fronts: fused tail
          if (L.cnt > 0) h->fac.push_back(L);
        }
        if (pos != act.size()) return fail(h, SMLU_ERR_ARG, "internal: panel classes");
      }
      // inverses of the diagonal tiles of the GEMM-form fronts (I - L_kk^-1, I - U_kk^-1)
      {
        L = Launch();
        L.kind = K_TRIINV;
        L.step = (int)t;
        L.off = (int64_t)ilist.size();
        for (auto s : act) {
          if (!gform(s) || fuse_inv) continue;   // fused into the panel launch
          ilist.push_back((int32_t)s);
          ilist.push_back((int32_t)slot_of(s, t % (h->ob / h->hsn[s].nb)));
        }
        L.cnt = ((int64_t)ilist.size() - L.off) / 2;
        if (L.cnt > 0) h->fac.push_back(L);
      }
      // row swaps inside the outer block (the other columns get them at the end of the block)
      {
        L = Launch();
        L.kind = K_LASWP;
        L.step = (int)t;
        L.off = (int64_t)st_tasks.size();
        int64_t wg = 0;
        for (auto s : act) {
          const SNode& r = h->hsn[s];
          int64_t kb = t * r.nb, w = std::min<int64_t>(r.nb, r.ns - kb);
          int64_t ostart = (kb / h->ob) * h->ob, oend = std::min<int64_t>(r.ns, ostart + h->ob);
          int64_t ncol = oend - ostart - w;
          if (ncol <= 0 || (fuse_panel && gform(s))) continue;   // fused panels swap these rows themselves
          st_tasks.push_back(SwapTask{(int32_t)s, (int32_t)kb, 1, (int32_t)slot_of(s, t % (h->ob / r.nb)),
                                      (int32_t)ostart, (int32_t)oend, (int32_t)kb, (int32_t)(kb + w), wg});
          wg += (ncol + 63) / 64;
        }
        L.cnt = (int64_t)st_tasks.size() - L.off;
        L.nwg = wg;
        if (wg > 0) h->fac.push_back(L);
      }
      {
        Launch T;
        T.kind = K_STEPTRSM;
        T.step = (int)t;
        T.off = (int64_t)ft.size();
        int64_t wgU = 0, W = 32, ntri = 0;
        for (auto s : act) {
          if (gform(s)) continue;
          ++ntri;
          const SNode& r = h->hsn[s];
          int64_t kb = t * r.nb, w = std::min<int64_t>(r.nb, r.ns - kb);
          int64_t ostart = (kb / h->ob) * h->ob, oend = std::min<int64_t>(r.ns, ostart + h->ob);
          ft.push_back(FrontTile{(int32_t)s, (int32_t)kb, wgU});
          wgU += (oend - kb - w + 255) / 256;
          W = std::max<int64_t>(W, w);
        }
        T.cnt = ntri;
        T.nwg = wgU;
        T.off2 = (int64_t)ft.size();
        int64_t wgL = 0;
        for (auto s : act) {
          if (gform(s)) continue;
          const SNode& r = h->hsn[s];
          int64_t M = (int64_t)r.ns + r.nu, kb = t * r.nb, w = std::min<int64_t>(r.nb, r.ns - kb);
          int64_t R = r.mode == 1 ? r.ns - kb : w;
          ft.push_back(FrontTile{(int32_t)s, (int32_t)kb, wgL});
          wgL += (M - kb - R + 255) / 256;
        }
        T.cnt2 = ntri;
        T.nwg2 = wgL;
        T.aux = W;
        if (wgU + wgL > 0) h->fac.push_back(T);
      }
      // GEMM-form step TRSM of the blocked fronts, in place (R = rows the panel finished:
      // w for diagonal-tile panels, every fully-summed row for full-candidate panels):
      //   U rows [kb, kb+w) x columns [kb+w, oend):  C - (I - L_kk^-1) C = L_kk^-1 C
      //   L rows [kb+R, M) x columns [kb, kb+w):     C - C (I - U_kk^-1) = C U_kk^-1 (+ growth)
      {
        std::vector<GemmTask> cand;
        std::vector<int64_t> tp;
        for (auto s : act) {
          if (!gform(s)) continue;
          const SNode& r = h->hsn[s];
          int64_t M = (int64_t)r.ns + r.nu, kb = t * r.nb, w = std::min<int64_t>(r.nb, r.ns - kb);
          int64_t ostart = (kb / h->ob) * h->ob, oend = std::min<int64_t>(r.ns, ostart + h->ob);
          const int64_t slot = slot_of(s, t % (h->ob / r.nb));
          if (oend - kb - w > 0) {
            GemmTask g{};
            g.B = g.C = store + r.Loff + (kb + w) * M + kb;
            g.m = (int)w; g.n = (int)(oend - kb - w); g.k = (int)w;
            g.lda = 64; g.ldb = (int)M; g.ldc = (int)M;
            cand.push_back(g);
            tp.push_back(tinv_slot_off(slot, false) * 2);
          }
          const int64_t R = r.mode == 1 ? r.ns - kb : w;   // rows the panel already finished
          if (M - kb - R > 0) {
            GemmTask g{};
            g.A = g.C = store + r.Loff + kb * M + kb + R;
            g.m = (int)(M - kb - R); g.n = (int)w; g.k = (int)w;
            g.lda = (int)M; g.ldb = 64; g.ldc = (int)M;
            g.gsid = (int32_t)s;
            cand.push_back(g);
            tp.push_back(tinv_slot_off(slot, true) * 2 + 1);
          }
        }
        add_gemm_launch(cand, 0.0, (int)t, K_TRSML, &tp);
      }
      // inner trailing update: rows [kb+w, M) x columns [kb+w, oend) of the outer block
      {
        std::vector<GemmTask> cand;
        double fl = 0;
        for (auto s : act) {
          const SNode& r = h->hsn[s];
          int64_t M = (int64_t)r.ns + r.nu, kb = t * r.nb, w = std::min<int64_t>(r.nb, r.ns - kb);
          int64_t ostart = (kb / h->ob) * h->ob, oend = std::min<int64_t>(r.ns, ostart + h->ob);
          int64_t m1 = M - kb - w, n1 = oend - kb - w;
          if (m1 > 0 && n1 > 0) {
            GemmTask g{};
            g.A = store + r.Loff + kb * M + kb + w;
            g.B = store + r.Loff + (kb + w) * M + kb;
            g.C = store + r.Loff + (kb + w) * M + kb + w;
            g.m = (int)m1; g.n = (int)n1; g.k = (int)w;
            g.lda = (int)M; g.ldb = (int)M; g.ldc = (int)M;
            cand.push_back(g);
            fl += 2.0 * m1 * n1 * w;
          }
        }
        add_gemm_launch(cand, fl, (int)t);
      }
      // end of an outer block [ostart, oend): deferred row swaps on the columns outside it, the
      // U rows of the block right of it, and the trailing update with k = oend - ostart
      std::vector<int64_t> fin_all;
      for (auto s : act) {
        const SNode& r = h->hsn[s];
        int64_t kb = t * r.nb, w = std::min<int64_t>(r.nb, r.ns - kb);
        int64_t ostart = (kb / h->ob) * h->ob, oend = std::min<int64_t>(r.ns, ostart + h->ob);
        if (kb + w == oend) fin_all.push_back(s);
      }
      if (fin_all.empty()) continue;
      {
        L = Launch();
        L.kind = K_LASWP;
        L.step = (int)t;
        L.off = (int64_t)st_tasks.size();
        int64_t wg = 0;
        for (auto s : fin_all) {
          const SNode& r = h->hsn[s];
          int64_t M = (int64_t)r.ns + r.nu, kb = t * r.nb;
          int64_t ostart = (kb / h->ob) * h->ob, oend = std::min<int64_t>(r.ns, ostart + h->ob);
          int64_t ncol = M - (oend - ostart);
          if (ncol <= 0) continue;
          st_tasks.push_back(SwapTask{(int32_t)s, (int32_t)ostart, (int32_t)((oend - ostart + r.nb - 1) / r.nb),
                                      (int32_t)slot_of(s, (ostart % h->ob) / r.nb), 0, (int32_t)M, (int32_t)ostart,
                                      (int32_t)oend, wg});
          wg += (ncol + 63) / 64;
        }
        L.cnt = (int64_t)st_tasks.size() - L.off;
        L.nwg = wg;
        if (wg > 0) h->fac.push_back(L);
      }
      // End of an outer block: its U rows on every column right of it (sub-panel by sub-panel,
      // k_urows or GEMM-form TRSM), then the trailing update with k = OB width
      struct URows {
        int64_t s, ob0, ob1, c0, c1;   // OB rows [ob0, ob1); L-panel columns [c0, c1); + U12 if u12
        bool u12;
      };
      // TRSM of the U rows of a set of OBs (one per front), sub-panel by sub-panel: L_uu^-1 C in
      // place on the given columns, then the rows below the sub-panel inside the OB
      auto urows = [&](const std::vector<URows>& all_items) {
        // GEMM-form fronts: one fused k_urows launch (every column block runs the whole
        // sub-panel sequence); the others keep one launch pair per sub-panel
        std::vector<URows> items;
        {
          L = Launch();
          L.kind = K_UROWS;
          L.step = (int)t;
          L.off = (int64_t)ur_tasks.size();
          for (auto& it : all_items) {
            const SNode& r = h->hsn[it.s];
            if (!(fuse_urows && gform(it.s))) {
              items.push_back(it);
              continue;
            }
            const int64_t M = (int64_t)r.ns + r.nu;
            const int32_t slot0 = (int32_t)slot_of(it.s, (it.ob0 % h->ob) / r.nb);
            for (int64_t c = it.c0; c < it.c1; c += kUrowsCols)
              ur_tasks.push_back(URowTask{(int32_t)it.s, (int32_t)it.ob0, (int32_t)it.ob1, slot0, (int32_t)M,
                                          (int32_t)std::min<int64_t>(kUrowsCols, it.c1 - c), r.Loff + c * M});
            if (it.u12)
              for (int64_t c = 0; c < r.nu; c += kUrowsCols)
                ur_tasks.push_back(URowTask{(int32_t)it.s, (int32_t)it.ob0, (int32_t)it.ob1, slot0, r.ns,
                                            (int32_t)std::min<int64_t>(kUrowsCols, r.nu - c), r.Uoff + c * r.ns});
          }
          L.cnt = (int64_t)ur_tasks.size() - L.off;
          if (L.cnt > 0) h->fac.push_back(L);
        }
        int64_t nsub = 0;
        for (auto& it : items) nsub = std::max<int64_t>(nsub, (it.ob1 - it.ob0 + h->hsn[it.s].nb - 1) / h->hsn[it.s].nb);
        for (int64_t u = 0; u < nsub; ++u) {
          L = Launch();
          L.kind = K_TRSMU;
          L.step = (int)t;
          L.aux = 1;   // outer mode
          L.off = (int64_t)ft.size();
          int64_t wg = 0, cnt = 0;
          std::vector<GemmTask> cand, ctri;
          std::vector<int64_t> tp;
          double fl = 0;
          for (auto& it : items) {
            const int64_t s = it.s;
            const SNode& r = h->hsn[s];
            const int64_t M = (int64_t)r.ns + r.nu;
            const int64_t kbu = it.ob0 + u * r.nb;
            if (kbu >= it.ob1) continue;
            const int64_t wu = std::min<int64_t>(r.nb, it.ob1 - kbu);
            const int64_t n1 = it.c1 - it.c0;
            if (gform(s)) {   // U rows [kbu, kbu+wu) on the columns: L_uu^-1 C, in place
              const int64_t off = tinv_slot_off(slot_of(s, (kbu % h->ob) / r.nb), false) * 2;
              if (n1 > 0) {
                GemmTask g{};
                g.B = g.C = store + r.Loff + it.c0 * M + kbu;
                g.m = (int)wu; g.n = (int)n1; g.k = (int)wu;
                g.lda = 64; g.ldb = (int)M; g.ldc = (int)M;
                ctri.push_back(g);
                tp.push_back(off);
              }
              if (it.u12 && r.nu > 0) {
                GemmTask g{};
                g.B = g.C = store + r.Uoff + kbu;
                g.m = (int)wu; g.n = r.nu; g.k = (int)wu;
                g.lda = 64; g.ldb = r.ns; g.ldc = r.ns;
                ctri.push_back(g);
                tp.push_back(off);
              }
            } else {          // k_trsm_u: columns [oend, M) of the plain two-level scheme
              ft.push_back(FrontTile{(int32_t)s, (int32_t)kbu, wg});
              wg += (M - it.c0 + 255) / 256;
              ++cnt;
            }
            // rows below the sub-panel inside the OB: [kbu+wu, ob1) x the columns
            const int64_t m = it.ob1 - kbu - wu;
            if (m > 0) {
              if (n1 > 0) {
                GemmTask g{};
                g.A = store + r.Loff + kbu * M + kbu + wu;
                g.B = store + r.Loff + it.c0 * M + kbu;
                g.C = store + r.Loff + it.c0 * M + kbu + wu;
                g.m = (int)m; g.n = (int)n1; g.k = (int)wu;
                g.lda = (int)M; g.ldb = (int)M; g.ldc = (int)M;
                cand.push_back(g);
                fl += 2.0 * m * n1 * wu;
              }
              if (it.u12 && r.nu > 0) {
                GemmTask g{};
                g.A = store + r.Loff + kbu * M + kbu + wu;
                g.B = store + r.Uoff + kbu;
                g.C = store + r.Uoff + kbu + wu;
                g.m = (int)m; g.n = r.nu; g.k = (int)wu;
                g.lda = (int)M; g.ldb = r.ns; g.ldc = r.ns;
                cand.push_back(g);
                fl += 2.0 * m * (double)r.nu * wu;
              }
            }
          }
          L.cnt = cnt;
          L.nwg = wg;
          if (wg > 0) h->fac.push_back(L);
          add_gemm_launch(ctri, 0.0, (int)t, K_TRSML, &tp);
          add_gemm_launch(cand, fl, (int)t, K_GEMMU);
        }
      };
      // C(rows [r0, r1) x L-panel columns [c0, c1) (+ U12 when u12)) -= L(rows, [k0, k1)) U([k0, k1), cols)
      auto rank_update = [&](int64_t s, int64_t r0, int64_t r1, int64_t c0, int64_t c1, bool u12, int64_t k0,
                             int64_t k1, std::vector<GemmTask>& cand, double& fl) {
        const SNode& r = h->hsn[s];
        const int64_t M = (int64_t)r.ns + r.nu, kk = k1 - k0;
        if (r1 > r0 && c1 > c0 && kk > 0) {
          GemmTask g{};
          g.A = store + r.Loff + k0 * M + r0;
          g.B = store + r.Loff + c0 * M + k0;
          g.C = store + r.Loff + c0 * M + r0;
          g.m = (int)(r1 - r0); g.n = (int)(c1 - c0); g.k = (int)kk;
          g.lda = (int)M; g.ldb = (int)M; g.ldc = (int)M;
          cand.push_back(g);
          fl += 2.0 * (double)(r1 - r0) * (double)(c1 - c0) * kk;
        }
        const int64_t ru1 = std::min<int64_t>(r1, r.ns);   // U12 rows live above ns
        if (u12 && r.nu > 0 && ru1 > r0 && kk > 0) {
          GemmTask g{};
          g.A = store + r.Loff + k0 * M + r0;
          g.B = store + r.Uoff + k0;
          g.C = store + r.Uoff + r0;
          g.m = (int)(ru1 - r0); g.n = r.nu; g.k = (int)kk;
          g.lda = (int)M; g.ldb = r.ns; g.ldc = r.ns;
          cand.push_back(g);
          fl += 2.0 * (double)(ru1 - r0) * (double)r.nu * kk;
        }
      };
      std::vector<URows> items;
      std::vector<GemmTask> c1;
      double fl1 = 0;
      for (auto s : fin_all) {
        const SNode& r = h->hsn[s];
        const int64_t kb = t * r.nb, M = (int64_t)r.ns + r.nu;
        const int64_t ostart = (kb / h->ob) * h->ob, oend = std::min<int64_t>(r.ns, ostart + h->ob);
        if (oend == M) continue;   // nothing right of the block
        items.push_back(URows{s, ostart, oend, oend, r.ns, true});
        rank_update(s, oend, M, oend, r.ns, false, ostart, oend, c1, fl1);
        rank_update(s, oend, r.ns, oend, oend, true, ostart, oend, c1, fl1);   // U12 rows only
      }
      urows(items);
      add_gemm_launch(c1, fl1, (int)t, K_GEMMO);
    }
    // F22 -= L21 * U12 for the blocked fronts of this level
    {
      std::vector<GemmTask> cand;
      double fl = 0;
      for (auto s : big) {
        const SNode& r = h->hsn[s];
        if (r.nu == 0) continue;
        int64_t M = (int64_t)r.ns + r.nu;
        GemmTask g{};
        g.A = store + r.Loff + r.ns;
        g.B = store + r.Uoff;
        g.C = scratch + r.Foff;
        g.m = r.nu; g.n = r.nu; g.k = r.ns;
        g.lda = (int)M; g.ldb = r.ns; g.ldc = r.nu;
        cand.push_back(g);
        fl += 2.0 * r.nu * (double)r.nu * r.ns;
      }
      add_gemm_launch(cand, fl, -1);
    }
    // the shared front of this level (multi-GPU): for each pivot block, its owner runs the inner
    // steps (64-column panels with diagonal-tile pivoting, tile inverses, in-block swaps, GEMM-form
    // triangular solves, in-block updates) on its copy, broadcasts the factored block (L rows
    // [ob, M), tile inverses, swap lists, rowperm) to the group, and every member applies it to
    // the column blocks it owns: deferred swaps, U rows (GEMM-form TRSM per sub-panel), the rows
    // below each sub-panel, and the trailing update (k = block width) down to the F22 rows
    for (const int32_t t : dfront[l]) {
      const SNode& fr = h->hsn[t];
      const int64_t ns = fr.ns, nu = fr.nu, M = ns + nu;
      const int64_t np = P.npblk(t);
      std::vector<size_t> mine;
      for (size_t i = 0; i < Y.blocks.size(); ++i)
        if (Y.blocks[i].s == t) mine.push_back(i);
      // look-ahead (depth 1, SMLU_DIST_LOOKAHEAD=1): the owner of pivot block b+1 applies block
      // b to block b+1 first, factors and broadcasts b+1, and only then applies b to its other
      // blocks (`pending`).  Off by default: the broadcast is a rendezvous (receivers post it
      // after their own trailing updates), so the deferred work only loads the next owner --
      // the schedule model projects 3.0x instead of 4.3x at 256^3 / 8 ranks with it on
      constexpr bool dist_lookahead = false;
      std::vector<Launch> pending;
      for (int64_t b = 0; b < np; ++b) {
        const int64_t ob = P.blk_c0(t, b), oe = P.blk_c1(t, b), w = oe - ob;
        const int64_t nsub = (w + 63) / 64;
        const int32_t o = P.blk_owner(t, b);
        const bool own = o == h->rank;
        int32_t bn = -1;
        double* Lb = nullptr;
        if (own) {
          bn = blknode[blkmap.at((int64_t)t * 1048576 + b)];
          Lb = store + h->hsn[bn].Loff;
          for (int64_t kb = ob; kb < oe; kb += 64) {
            const int64_t wk = std::min<int64_t>(64, oe - kb);
            const int step = (int)(kb / 64);
            const int32_t u = (int32_t)((kb - ob) / 64);
            Launch Q;
            Q.kind = K_PANEL;
            Q.step = step;
            Q.off = (int64_t)ilist.size();
            ilist.push_back(bn);
            ilist.push_back(u);
            Q.cnt = 1;
            Q.nwg = wk;
            Q.aux2 = 64;
            h->fac.push_back(Q);
            Q = Launch();
            Q.kind = K_TRIINV;
            Q.step = step;
            Q.off = (int64_t)ilist.size();
            ilist.push_back(bn);
            ilist.push_back(u);
            Q.cnt = 1;
            h->fac.push_back(Q);
            if (oe - ob - wk > 0) {
              Q = Launch();
              Q.kind = K_LASWP;
              Q.step = step;
              Q.off = (int64_t)st_tasks.size();
              st_tasks.push_back(SwapTask{bn, (int32_t)kb, 1, u, (int32_t)ob, (int32_t)oe, (int32_t)kb,
                                          (int32_t)(kb + wk), 0});
              Q.cnt = 1;
              Q.nwg = (oe - ob - wk + 63) / 64;
              h->fac.push_back(Q);
            }
            std::vector<GemmTask> cand;
            std::vector<int64_t> tp;
            if (oe - kb - wk > 0) {
              GemmTask g{};
              g.B = g.C = Lb + (kb + wk) * M + kb;
              g.m = (int)wk; g.n = (int)(oe - kb - wk); g.k = (int)wk;
              g.lda = 64; g.ldb = (int)M; g.ldc = (int)M;
              cand.push_back(g);
              tp.push_back(tinv_slot_off(u, false) * 2);
            }
            if (M - kb - wk > 0) {
              GemmTask g{};
              g.A = g.C = Lb + kb * M + kb + wk;
              g.m = (int)(M - kb - wk); g.n = (int)wk; g.k = (int)wk;
              g.lda = (int)M; g.ldb = 64; g.ldc = (int)M;
              g.gsid = bn;
              cand.push_back(g);
              tp.push_back(tinv_slot_off(u, true) * 2 + 1);
            }
            add_gemm_launch(cand, 0.0, step, K_TRSML, &tp);
            if (M - kb - wk > 0 && oe - kb - wk > 0) {
              GemmTask g{};
              g.A = Lb + kb * M + kb + wk;
              g.B = Lb + (kb + wk) * M + kb;
              g.C = Lb + (kb + wk) * M + kb + wk;
              g.m = (int)(M - kb - wk); g.n = (int)(oe - kb - wk); g.k = (int)wk;
              g.lda = (int)M; g.ldb = (int)M; g.ldc = (int)M;
              std::vector<GemmTask> c1{g};
              add_gemm_launch(c1, 2.0 * g.m * (double)g.n * wk, step);
            }
          }
        }
        // broadcast: [L rows [ob, M) x w, ld M-ob | tile inverses | swap lists | rowperm]
        const int64_t lbytes = 8 * (M - ob) * w, tbytes = 8 * nsub * 8192;
        const int64_t swbytes = 4 * nsub * kSwapStride, rpbytes = 4 * w;
        {
          CommOp op;
          op.type = 1;
          op.root = o;
          op.grp = P.group[t];
          op.bytes = lbytes + tbytes + swbytes + rpbytes;
          if (own) {
            op.bbase = 4;
            for (int64_t c = ob; c < oe; ++c)
              op.pack.push_back(HSeg{0, 8 * (h->hsn[bn].Loff + c * M + ob), 4, 8 * (c - ob) * (M - ob), 8 * (M - ob)});
            op.pack.push_back(HSeg{7, 0, 4, lbytes, tbytes});
            op.pack.push_back(HSeg{8, 0, 4, lbytes + tbytes, swbytes});
            op.pack.push_back(HSeg{9, 4 * (fr.first + ob), 4, lbytes + tbytes + swbytes, rpbytes});
          } else {
            op.bbase = 6;
            op.unpack.push_back(HSeg{6, lbytes + tbytes, 8, 0, swbytes});
            op.unpack.push_back(HSeg{6, lbytes + tbytes + swbytes, 9, 4 * (fr.first + ob), rpbytes});
          }
          add_comm(h->fac, h->fac_seg, h->fac_comm, std::move(op));
        }
        for (auto& q : pending) h->fac.push_back(q);   // the previous block's deferred updates
        pending.clear();
        const double* bc = h->bcbuf.p;
        const int64_t ldL = own ? M : M - ob;
        auto Lsrc = [&](int64_t row, int64_t col) -> const double* {
          return own ? Lb + col * M + row : bc + (col - ob) * (M - ob) + (row - ob);
        };
        // deferred row swaps on this rank's other blocks (left and right)
        {
          Launch Q;
          Q.kind = K_LASWP;
          Q.off = (int64_t)st_tasks.size();
          int64_t wg = 0;
          for (size_t i : mine) {
            const RankLayout::Blk& T = Y.blocks[i];
            if (T.b == b) continue;
            st_tasks.push_back(SwapTask{blknode[i], (int32_t)ob, (int32_t)nsub, 0, (int32_t)T.c0, (int32_t)T.c1,
                                        (int32_t)T.c1, (int32_t)T.c1, wg});
            wg += (T.c1 - T.c0 + 63) / 64;
          }
          Q.cnt = (int64_t)st_tasks.size() - Q.off;
          Q.nwg = wg;
          if (wg > 0) h->fac.push_back(Q);
        }
        // target blocks right of this one: (node, columns, pivot block?) and their row pointers
        struct Tgt { int32_t node; int64_t c0, c1; bool piv; };
        std::vector<Tgt> right_all, right;
        for (size_t i : mine) {
          const RankLayout::Blk& T = Y.blocks[i];
          if (T.c0 >= oe) right_all.push_back({blknode[i], T.c0, T.c1, T.c0 < ns});
        }
        // this rank owns pivot block b+1 (look-ahead): block b+1 first, the rest deferred
        const bool ahead = dist_lookahead && b + 1 < np && P.blk_owner(t, b + 1) == h->rank;
        for (int pass = 0; pass < 2; ++pass) {
        if (!ahead && pass == 1) break;
        right.clear();
        for (const Tgt& T : right_all)
          if (!ahead || (pass == 0) == (T.c0 == P.blk_c0(t, b + 1))) right.push_back(T);
        if (right.empty()) continue;
        std::vector<Launch> saved;
        if (ahead && pass == 1) saved.swap(h->fac);   // emit the deferred part into `pending`
        auto trow = [&](const Tgt& T, int64_t row) -> double* {   // rows < ns of the target's first column
          const SNode& q = h->hsn[T.node];
          return T.piv ? store + q.Loff + T.c0 * M + row : store + q.Uoff + (T.c0 - ns) * ns + row;
        };
        for (int64_t u = 0; u < nsub; ++u) {
          const int64_t kbu = ob + 64 * u, wu = std::min<int64_t>(64, oe - kbu);
          std::vector<GemmTask> ctri, cand;
          std::vector<int64_t> tp;
          double fl = 0;
          for (const Tgt& T : right) {
            const int ldt = (int)(T.piv ? M : ns);
            GemmTask g{};
            g.B = g.C = trow(T, kbu);
            g.m = (int)wu; g.n = (int)(T.c1 - T.c0); g.k = (int)wu;
            g.lda = 64; g.ldb = ldt; g.ldc = ldt;
            if (own) tp.push_back(tinv_slot_off(u, false) * 2);
            else { g.A = bc + (M - ob) * w + u * 8192; tp.push_back(-1); }
            ctri.push_back(g);
            const int64_t m = oe - kbu - wu;
            if (m > 0) {
              GemmTask q{};
              q.A = Lsrc(kbu + wu, kbu);
              q.B = trow(T, kbu);
              q.C = trow(T, kbu + wu);
              q.m = (int)m; q.n = (int)(T.c1 - T.c0); q.k = (int)wu;
              q.lda = (int)ldL; q.ldb = ldt; q.ldc = ldt;
              cand.push_back(q);
              fl += 2.0 * m * (double)(T.c1 - T.c0) * wu;
            }
          }
          add_gemm_launch(ctri, 0.0, (int)(kbu / 64), K_TRSML, &tp);
          add_gemm_launch(cand, fl, (int)(kbu / 64), K_GEMMU);
        }
        {
          std::vector<GemmTask> cand;
          double fl = 0;
          for (const Tgt& T : right) {
            const int64_t nc = T.c1 - T.c0;
            if (T.piv) {
              if (M - oe <= 0) continue;
              GemmTask g{};
              g.A = Lsrc(oe, ob);
              g.B = trow(T, ob);
              g.C = trow(T, oe);
              g.m = (int)(M - oe); g.n = (int)nc; g.k = (int)w;
              g.lda = (int)ldL; g.ldb = (int)M; g.ldc = (int)M;
              cand.push_back(g);
              fl += 2.0 * (M - oe) * (double)nc * w;
            } else {
              if (ns - oe > 0) {
                GemmTask g{};
                g.A = Lsrc(oe, ob);
                g.B = trow(T, ob);
                g.C = trow(T, oe);
                g.m = (int)(ns - oe); g.n = (int)nc; g.k = (int)w;
                g.lda = (int)ldL; g.ldb = (int)ns; g.ldc = (int)ns;
                cand.push_back(g);
                fl += 2.0 * (ns - oe) * (double)nc * w;
              }
              if (nu > 0) {
                const SNode& q = h->hsn[T.node];
                GemmTask g{};
                g.A = Lsrc(ns, ob);
                g.B = trow(T, ob);
                g.C = scratch + q.Foff + (T.c0 - ns) * nu;
                g.m = (int)nu; g.n = (int)nc; g.k = (int)w;
                g.lda = (int)ldL; g.ldb = (int)ns; g.ldc = (int)nu;
                cand.push_back(g);
                fl += 2.0 * nu * (double)nc * w;
              }
            }
          }
          add_gemm_launch(cand, fl, (int)(ob / 64), K_GEMMO);
        }
        if (ahead && pass == 1) {
          pending.swap(h->fac);
          h->fac.swap(saved);
        }
        }
      }
      for (auto& q : pending) h->fac.push_back(q);
      pending.clear();
    }
  }
  // solves: per level, small fronts by one workgroup each; large fronts (ns > kSolveBigNs)
  // gather + one launch per 64-column block with 256-row chunks per workgroup
  h->fwd.clear();
  h->bwd.clear();
  std::vector<std::vector<Launch>> bwd_levels;
  auto node_of = [&](int64_t s, int64_t b) { return blknode[blkmap.at(s * 1048576 + b)]; };
  auto tri_steps = [&](bool upper, int32_t node, int64_t ob, int64_t oe, std::vector<Launch>& out) {
    const SNode& r = h->hsn[node];
    const int64_t M = (int64_t)r.ns + r.nu, nbs = (r.ns + 63) / 64;
    std::vector<int64_t> jbs;
    for (int64_t jb = ob; jb < oe; jb += 64) jbs.push_back(jb);
    if (upper) std::reverse(jbs.begin(), jbs.end());
    for (int64_t jb : jbs) {
      Launch F;
      F.kind = upper ? K_TRIB : K_TRIF;
      F.step = (int)(upper ? nbs - 1 - jb / 64 : jb / 64);
      F.off = (int64_t)ft.size();
      const int64_t bw = std::min<int64_t>(64, r.ns - jb);
      const int64_t wg = upper ? std::max<int64_t>(1, (jb + 255) / 256) : std::max<int64_t>(1, (M - jb - bw + 255) / 256);
      ft.push_back(FrontTile{node, 0, 0});
      F.cnt = 1;
      F.nwg = wg;
      out.push_back(F);
    }
  };
  // one vector segment of vbuf (doubles [off, off+cnt)) from rank a to rank b, in place
  auto vhop = [&](std::vector<Launch>& seq, std::vector<size_t>& seg, std::vector<int>& cm, int32_t a, int32_t b,
                  int64_t off, int64_t cnt) {
    if (a == b || cnt <= 0 || (h->rank != a && h->rank != b)) return;
    CommOp op;
    const int pi = op.at(h->rank == a ? b : a);
    if (h->rank == a) { op.sbase[pi] = 2; op.soff[pi] = 8 * off; op.sbytes[pi] = 8 * cnt; }
    else { op.rbase[pi] = 2; op.roff[pi] = 8 * off; op.rbytes[pi] = 8 * cnt; }
    add_comm(seq, seg, cm, std::move(op));
  };
  auto holder = [&](int64_t c) { return P.dist(c) ? P.blk_owner(c, P.npblk(c) - 1) : P.owner[c]; };
  constexpr bool no_tiny = false, no_micro = false;
  // large fronts: one sync-free sweep launch per level and direction (default) or one launch per
  // 64-column block (SMLU_SOLVE_STEPS=1, the previous schedule)
  const bool sweep_solve = !tn.solve_steps;
  int64_t ssync_n = 0, ntick = 0;   // flags and ticket counters of the sweep launches
  constexpr int64_t big_work = kSolveBigWork;
  for (int l = 0; l < P.nlevels; ++l) {
    std::vector<int64_t> tiny, small, bigs;
    for (int64_t k = LP[l]; k < LP[l + 1]; ++k) {
      int64_t s = LS[k];
      const SNode& r = h->hsn[s];
      const bool big = r.ns > kSolveBigNs || (int64_t)r.ns * ((int64_t)r.ns + r.nu) > big_work;
      const bool tiny_front = (int64_t)r.ns + r.nu <= kSolveTinyM && r.ns <= 64 && !no_tiny;
      (big ? bigs : tiny_front ? tiny : small).push_back(s);
    }
    std::vector<Launch> bl;
    // tiny fronts: one wave per front; micro fronts (M <= 8) eight per wave for a single rhs
    for (int micro = 1; micro >= 0; --micro) {
      Launch L;
      L.kind = K_FWDT;
      L.aux = micro;
      L.off = (int64_t)ilist.size();
      for (auto s : tiny)
        if ((P.M(s) <= kSolveMicroM && !no_micro) == (micro == 1)) ilist.push_back((int32_t)s);
      L.cnt = (int64_t)ilist.size() - L.off;
      if (L.cnt == 0) continue;
      h->fwd.push_back(L);
      L.kind = K_BWDT;
      bl.push_back(L);
    }
    if (!small.empty()) {
      Launch L;
      L.kind = K_FWD;
      L.off = (int64_t)ilist.size();
      for (auto s : small) ilist.push_back((int32_t)s);
      L.cnt = (int64_t)small.size();
      h->fwd.push_back(L);
      L.kind = K_BWD;
      bl.push_back(L);
    }
    if (!bigs.empty()) {
      // gather: one thread per front row pulls its own value and the children's contributions (in
      // child order) -- k_fwd_pull; pull lists per front row: gptr (CSR, relative to the front's
      // block) -> gent (vbuf index of each contribution)
      Launch L;
      L.kind = K_FWDP;
      L.off = (int64_t)ft.size();
      int64_t wgp = 0;
      for (auto s : bigs) {
        const SNode& r = h->hsn[s];
        const int64_t M = (int64_t)r.ns + r.nu;
        ft.push_back(FrontTile{(int32_t)s, (int32_t)gptr.size(), wgp});
        wgp += (M + 255) / 256;
        std::vector<int32_t> cnt(M + 1, 0);
        for (int c = r.chbeg; c < r.chend; ++c) {
          const SNode& ch = h->hsn[P.ch_list[c]];
          const int32_t* rm = P.relmap.data() + ch.rowptr;
          for (int32_t k = 0; k < ch.nu; ++k) ++cnt[rm[k] + 1];
        }
        for (int64_t t = 0; t < M; ++t) cnt[t + 1] += cnt[t];
        const int64_t base = (int64_t)gent.size();
        for (int64_t t = 0; t <= M; ++t) gptr.push_back((int32_t)(base + cnt[t]));
        gent.resize(base + cnt[M]);
        for (int c = r.chbeg; c < r.chend; ++c) {
          const SNode& ch = h->hsn[P.ch_list[c]];
          const int32_t* rm = P.relmap.data() + ch.rowptr;
          for (int32_t k = 0; k < ch.nu; ++k) gent[base + cnt[rm[k]]++] = (int32_t)(ch.voff + ch.ns + k);
        }
        if ((int64_t)gptr.size() >= INT32_MAX || (int64_t)gent.size() >= INT32_MAX || r.voff + M >= INT32_MAX)
          return fail(h, SMLU_ERR_ALLOC, "solve gather lists exceed 32-bit indices");
      }
      L.cnt = (int64_t)bigs.size();
      L.nwg = wgp;
      h->fwd.push_back(L);
      int64_t nb = 0;
      for (auto s : bigs) nb = std::max<int64_t>(nb, (h->hsn[s].ns + 63) / 64);
      // backward: U12 product first
      Launch U;
      U.kind = K_BWDU;
      U.off = (int64_t)ft.size();
      int64_t wg = 0;
      for (auto s : bigs) {
        ft.push_back(FrontTile{(int32_t)s, 0, wg});
        wg += (h->hsn[s].ns + 63) / 64;   // k_bwd_u12: 64 rows per workgroup
      }
      U.cnt = (int64_t)bigs.size();
      U.nwg = wg;
      if (sweep_solve) {   // one sync-free sweep launch per direction (k_tri_sweep)
        Launch F, B;
        F.kind = K_SWEEPF;
        B.kind = K_SWEEPB;
        F.off = (int64_t)ft.size();
        F.aux = ssync_n;
        F.aux2 = ntick++;
        int64_t wf = 0;
        int32_t fb = 0;
        for (auto s : bigs) {
          const SNode& r = h->hsn[s];
          ft.push_back(FrontTile{(int32_t)s, fb, wf});
          wf += ((int64_t)r.ns + r.nu + 64 * kSweepWK - 1) / (64 * kSweepWK);
          fb += (r.ns + 63) / 64;
        }
        F.cnt = (int64_t)bigs.size();
        F.nwg = wf;
        ssync_n += fb;
        h->fwd.push_back(F);
        B.off = (int64_t)ft.size();
        B.aux = ssync_n;
        B.aux2 = ntick++;
        int64_t wb = 0;
        fb = 0;
        for (auto s : bigs) {
          const SNode& r = h->hsn[s];
          const int64_t nbs = (r.ns + 63) / 64;
          ft.push_back(FrontTile{(int32_t)s, fb, wb});
          wb += (nbs + kSweepWK - 1) / kSweepWK;
          fb += (int32_t)nbs;
        }
        B.cnt = (int64_t)bigs.size();
        B.nwg = wb;
        ssync_n += fb;
        bl.push_back(U);
        bl.push_back(B);
        bwd_levels.push_back(bl);
        goto shared_fronts;
      }
      std::vector<Launch> bsteps;
      for (int64_t t = 0; t < nb; ++t) {
        Launch F, B;
        F.kind = K_TRIF;
        B.kind = K_TRIB;
        F.step = B.step = (int)t;
        F.off = (int64_t)ft.size();
        int64_t wf = 0, cnt = 0;
        for (auto s : bigs) {
          const SNode& r = h->hsn[s];
          int64_t nbs = (r.ns + 63) / 64;
          if (t >= nbs) continue;
          int64_t jb = t * 64, bw = std::min<int64_t>(64, r.ns - jb), M = (int64_t)r.ns + r.nu;
          ft.push_back(FrontTile{(int32_t)s, 0, wf});
          wf += std::max<int64_t>(1, (M - jb - bw + 255) / 256);
          ++cnt;
        }
        F.cnt = cnt;
        F.nwg = wf;
        h->fwd.push_back(F);
        B.off = (int64_t)ft.size();
        int64_t wb = 0;
        cnt = 0;
        for (auto s : bigs) {
          const SNode& r = h->hsn[s];
          int64_t nbs = (r.ns + 63) / 64;
          if (t >= nbs) continue;
          int64_t jb = (nbs - 1 - t) * 64;
          ft.push_back(FrontTile{(int32_t)s, 0, wb});
          wb += std::max<int64_t>(1, (jb + 255) / 256);
          ++cnt;
        }
        B.cnt = cnt;
        B.nwg = wb;
        bsteps.push_back(B);
      }
      bl.push_back(U);
      for (auto& b : bsteps) bl.push_back(b);
    }
    bwd_levels.push_back(bl);
  shared_fronts:
    // forward solve of the shared front: the children's update vectors go to the first block's
    // owner, which gathers the front vector; the vector then follows the pivot blocks' owners
    // (shared fronts of this level, in front order on every rank)
    for (const int32_t t : dfront[l]) {
      const int64_t np = P.npblk(t), M = P.M(t);
      const int64_t tv = h->hsn[t].voff;
      const int32_t o0 = P.blk_owner(t, 0);
      {
        CommOp op;
        std::vector<std::vector<int64_t>> kids(h->nranks);
        for (int64_t e = P.ch_ptr[t]; e < P.ch_ptr[t + 1]; ++e) kids[holder(P.ch_list[e])].push_back(P.ch_list[e]);
        for (int32_t q = 0; q < h->nranks; ++q) {
          if (q == o0 || kids[q].empty()) continue;
          if (h->rank != q && h->rank != o0) continue;
          const int pi = op.at(h->rank == q ? o0 : q);
          int64_t acc = 0;
          for (int64_t c : kids[q]) {
            const int64_t off = 8 * (h->hsn[c].voff + P.ns(c)), nb8 = 8 * P.nu(c);
            if (h->rank == q) op.pack.push_back(HSeg{2, off, 4, acc, nb8});
            else op.unpack.push_back(HSeg{5, acc, 2, off, nb8});
            acc += nb8;
          }
          if (h->rank == q) op.sbytes[pi] = acc;
          else op.rbytes[pi] = acc;
        }
        // receive offsets: per peer contiguous in the receive staging
        int64_t racc = 0;
        for (size_t i = 0; i < op.peer.size(); ++i) {
          op.roff[i] = racc;
          racc += op.rbytes[i];
        }
        if (h->rank == o0) {   // unpack offsets were per peer from 0: shift by the peer's roff
          size_t k = 0;
          for (int32_t q = 0; q < h->nranks; ++q) {
            if (q == o0 || kids[q].empty()) continue;
            int64_t shift = 0;
            for (size_t i = 0; i < op.peer.size(); ++i)
              if (op.peer[i] == q) shift = op.roff[i];
            for (size_t j = 0; j < kids[q].size(); ++j) op.unpack[k++].so += shift;
          }
        }
        if (!op.peer.empty()) add_comm(h->fwd, h->fwd_seg, h->fwd_comm, std::move(op));
      }
      if (h->rank == o0) {
        Launch L;
        L.kind = K_FWDG;
        L.off = (int64_t)ilist.size();
        ilist.push_back(t);
        L.cnt = 1;
        h->fwd.push_back(L);
      }
      for (int64_t b = 0; b < np; ++b) {
        const int32_t o = P.blk_owner(t, b);
        const int64_t ob = P.blk_c0(t, b), oe = P.blk_c1(t, b);
        if (h->rank == o) tri_steps(false, node_of(t, b), ob, oe, h->fwd);
        if (b + 1 < np) vhop(h->fwd, h->fwd_seg, h->fwd_comm, o, P.blk_owner(t, b + 1), tv + oe, M - oe);
      }
    }
  }
  // backward, from the root level down; after each level holding a shared front (and at the
  // end) every rank shares the solution rows it computed since the previous exchange
  std::vector<std::vector<std::pair<int64_t, int64_t>>> pending_rows(h->nranks);   // per rank, since the last exchange
  std::vector<std::pair<int64_t, int64_t>> myrows;   // x rows (first, count) since the last exchange
  auto xbwd = [&]() {
    CommOp op;
    int64_t mine = 0;
    for (auto& rg : myrows) {
      op.pack.push_back(HSeg{3, 8 * rg.first, 4, 8 * mine, 8 * rg.second});
      mine += rg.second;
    }
    // every peer's rows, in its own order (the same enumeration on every rank)
    std::vector<std::vector<std::pair<int64_t, int64_t>>> theirs(h->nranks);
    theirs.swap(pending_rows);
    int64_t racc = 0;
    for (int32_t q = 0; q < h->nranks; ++q) {
      if (q == h->rank) continue;
      const int pi = op.at(q);
      op.soff[pi] = 0;
      op.sbytes[pi] = 8 * mine;
      op.roff[pi] = racc;
      int64_t cnt = 0;
      for (auto& rg : theirs[q]) {
        op.unpack.push_back(HSeg{5, racc + 8 * cnt, 3, 8 * rg.first, 8 * rg.second});
        cnt += rg.second;
      }
      op.rbytes[pi] = 8 * cnt;
      racc += 8 * cnt;
    }
    myrows.clear();
    add_comm(h->bwd, h->bwd_seg, h->bwd_comm, std::move(op));
  };
  (void)xbwd;
  for (int l = P.nlevels - 1; l >= 0; --l) {
    for (auto& L : bwd_levels[l]) h->bwd.push_back(L);
    if (h->nranks == 1) continue;
    // rows every rank computes at this level (global enumeration)
    for (int64_t k = P.lev_ptr[l]; k < P.lev_ptr[l + 1]; ++k) {
      const int64_t s = P.lev_sup[k];
      if (!P.dist(s)) {
        pending_rows[P.owner[s]].push_back({P.s_first[s], P.ns(s)});
        continue;
      }
      for (int64_t b = 0; b < P.npblk(s); ++b)
        pending_rows[P.blk_owner(s, b)].push_back({P.s_first[s] + P.blk_c0(s, b), P.blk_c1(s, b) - P.blk_c0(s, b)});
    }
    // (shared fronts of this level, in front order on every rank)
    for (const int32_t t : dfront[l]) {
      const int64_t np = P.npblk(t), nbk = np + P.nublk(t), ns = P.ns(t);
      const int64_t tv = h->hsn[t].voff;
      // the forward solve left y of each pivot block in x on the block's owner: the rank that
      // starts the backward chain collects all of them first
      const int32_t cs = nbk > np ? P.blk_owner(t, np) : P.blk_owner(t, np - 1);
      {
        CommOp op;
        const int64_t f0 = P.s_first[t];
        for (int32_t q = 0; q < h->nranks; ++q) {
          if (q == cs || (h->rank != q && h->rank != cs)) continue;
          int64_t acc = 0;
          std::vector<HSeg> segs;
          for (int64_t b = 0; b < np; ++b) {
            if (P.blk_owner(t, b) != q) continue;
            const int64_t o8 = 8 * (f0 + P.blk_c0(t, b)), nb8 = 8 * (P.blk_c1(t, b) - P.blk_c0(t, b));
            segs.push_back(h->rank == q ? HSeg{3, o8, 4, acc, nb8} : HSeg{5, acc, 3, o8, nb8});
            acc += nb8;
          }
          if (acc == 0) continue;
          const int pi = op.at(h->rank == q ? cs : q);
          if (h->rank == q) {
            op.sbytes[pi] = acc;
            for (auto& g : segs) op.pack.push_back(g);
          } else {
            op.rbytes[pi] = acc;
            for (auto& g : segs) op.unpack.push_back(g);
          }
        }
        if (h->rank == cs) {   // receive offsets per peer, shift the unpack copies
          int64_t racc = 0;
          size_t k = 0;
          for (size_t i = 0; i < op.peer.size(); ++i) {
            op.roff[i] = racc;
            int64_t left = op.rbytes[i];
            while (left > 0 && k < op.unpack.size()) {
              op.unpack[k].so += racc;
              left -= op.unpack[k].bytes;
              ++k;
            }
            racc += op.rbytes[i];
          }
        }
        if (!op.peer.empty()) add_comm(h->bwd, h->bwd_seg, h->bwd_comm, std::move(op));
      }
      int32_t prev = -1;
      bool first = true;
      for (int64_t ub = np; ub < nbk; ++ub) {   // U12 contributions, block by block
        const int32_t o = P.blk_owner(t, ub);
        if (prev >= 0) vhop(h->bwd, h->bwd_seg, h->bwd_comm, prev, o, tv, ns);
        if (h->rank == o) {
          Launch L;
          L.kind = K_BWDU12C;
          L.node = node_of(t, ub);
          L.aux = P.blk_c0(t, ub);
          L.aux2 = P.blk_c1(t, ub);
          L.cnt = first ? 1 : 0;
          h->bwd.push_back(L);
        }
        prev = o;
        first = false;
      }
      if (first) {   // no update columns: the chain starts from the solution rows of the front
        prev = P.blk_owner(t, np - 1);
        if (h->rank == prev) {
          Launch L;
          L.kind = K_VCOPY;
          L.node = t;
          h->bwd.push_back(L);
        }
      }
      for (int64_t b = np - 1; b >= 0; --b) {
        const int32_t o = P.blk_owner(t, b);
        const int64_t ob = P.blk_c0(t, b), oe = P.blk_c1(t, b);
        vhop(h->bwd, h->bwd_seg, h->bwd_comm, prev, o, tv, oe);
        if (h->rank == o) tri_steps(true, node_of(t, b), ob, oe, h->bwd);
        prev = o;
      }
    }
    for (auto& rg : pending_rows[h->rank]) myrows.push_back(rg);
    pending_rows[h->rank].clear();
    if (dlevel[l] || l == 0) xbwd();
  }

  h->nlaunch = (int64_t)h->fac.size();
  // upload
  HIPCHK(h->sn.upload(h->hsn.data(), h->hsn.size(), st));
  HIPCHK(h->ilist.upload(ilist.data(), ilist.size(), st));
  HIPCHK(h->xtasks.upload(xt.data(), xt.size(), st));
  HIPCHK(h->aents.upload(ae.data(), ae.size(), st));
  // batched right-hand sides (one GPU): the sweep's single chain wave per block would run the NR
  // chains one after another, so batches keep the per-64-column-block launches (k_tri_block: the
  // diagonal block solved by four chain waves for four right-hand sides at a time).  The same
  // per-block sequences (with the comm segments of fwd / bwd) re-run a solve whose sweep timed out.
  h->fwdm.clear();
  h->bwdm.clear();
  {
    auto expand = [&](const Launch& S, bool upper, std::vector<Launch>& out) {
      std::vector<int32_t> fr;
      for (int64_t i = S.off; i < S.off + S.cnt; ++i) fr.push_back(ft[i].s);
      int64_t nb = 0;
      for (auto s : fr) nb = std::max<int64_t>(nb, (h->hsn[s].ns + 63) / 64);
      for (int64_t t = 0; t < nb; ++t) {
        Launch F;
        F.kind = upper ? K_TRIB : K_TRIF;
        F.step = (int)t;
        F.off = (int64_t)ft.size();
        int64_t w = 0, cnt = 0;
        for (auto s : fr) {
          const SNode& r = h->hsn[s];
          const int64_t nbs = (r.ns + 63) / 64, M = (int64_t)r.ns + r.nu;
          if (t >= nbs) continue;
          const int64_t jb = upper ? (nbs - 1 - t) * 64 : t * 64, bw = std::min<int64_t>(64, r.ns - jb);
          ft.push_back(FrontTile{s, 0, w});
          w += upper ? std::max<int64_t>(1, (jb + 255) / 256) : std::max<int64_t>(1, (M - jb - bw + 255) / 256);
          ++cnt;
        }
        F.cnt = cnt;
        F.nwg = w;
        out.push_back(F);
      }
    };
    auto expand_all = [&](const std::vector<Launch>& in, const std::vector<size_t>& seg, bool upper,
                          std::vector<Launch>& out, std::vector<size_t>& oseg) {
      std::vector<size_t> at(in.size() + 1);
      for (size_t i = 0; i < in.size(); ++i) {
        at[i] = out.size();
        if (in[i].kind == (upper ? K_SWEEPB : K_SWEEPF)) expand(in[i], upper, out);
        else out.push_back(in[i]);
      }
      at[in.size()] = out.size();
      oseg.clear();
      for (size_t k : seg) oseg.push_back(at[std::min(k, in.size())]);
    };
    expand_all(h->fwd, h->fwd_seg, false, h->fwdm, h->fwdm_seg);
    expand_all(h->bwd, h->bwd_seg, true, h->bwdm, h->bwdm_seg);
  }
  HIPCHK(h->ftiles.upload(ft.data(), ft.size(), st));
  if (!gptr.empty()) {
    HIPCHK(h->gptr.upload(gptr.data(), gptr.size(), st));
    HIPCHK(h->gent.upload(gent.data(), gent.size(), st));
  }
  h->ssync_n = ssync_n;
  if (ssync_n > 0) {   // zeroed once per schedule: the sweeps never reset them (epochs, kernels_solve.hip)
    HIPCHK(h->ssync.alloc((size_t)ssync_n));
    HIPCHK(h->stick.alloc((size_t)ntick));
    HIPCHK(h->sxh.alloc((size_t)ssync_n * 64 * kMultiRhs));
    {   // hand-off slots start as the sweep's sentinel (kernels_solve.hip: k_tri_sweep)
      const long long sent = 0x7ff4dead5eed0001ll;
      double sv;
      std::memcpy(&sv, &sent, sizeof sv);
      HIPCHK(launch_fill(st, ssync_n * 64 * kMultiRhs, h->sxh.p, sv));
    }
    HIPCHK(hipMemsetAsync(h->ssync.p, 0, sizeof(int32_t) * ssync_n, st));
    HIPCHK(hipMemsetAsync(h->stick.p, 0, sizeof(unsigned long long) * ntick, st));
    HIPCHK(hipStreamSynchronize(st));
  }
  if (!h->sstatus.p) {
    HIPCHK(h->sstatus.alloc(1));
    HIPCHK(hipMemsetAsync(h->sstatus.p, 0, sizeof(int32_t), st));
  }
  h->sweep_spin = tn.sweep_spin;
  if (h->nranks > 1) max_list = std::max<int64_t>(max_list, dist_slots);
  if (!tinv_patch.empty() || h->nranks > 1) {   // operands in the tile-inverse slots: patch in the buffer address
    HIPCHK(h->tinv.alloc((size_t)max_list * 8192));
    for (auto& pt : tinv_patch) {
      const double* a = h->tinv.p + pt.second / 2;
      if (pt.second & 1) gt[pt.first].B = a;
      else gt[pt.first].A = a;
    }
  }
  HIPCHK(h->gtasks.upload(gt.data(), gt.size(), st));
  HIPCHK(h->stasks.upload(st_tasks.data(), st_tasks.size(), st));
  HIPCHK(h->urtasks.upload(ur_tasks.data(), ur_tasks.size(), st));
  HIPCHK(h->xcols.upload(xc.data(), xc.size(), st));
  HIPCHK(h->swaps.alloc((size_t)max_list * kSwapStride));
  HIPCHK(h->vbuf.alloc((size_t)std::max<int64_t>(voff, 1)));
  // communication steps: staging sizes, then every pack / unpack copy as a device descriptor
  if (!h->comm.empty()) {
    int64_t ss = 0, rs = 0, hs = 0, hr = 0;
    for (const CommOp& op : h->comm) {
      int64_t a = 0, b = 0, sa = 0, sb = 0;
      for (size_t i = 0; i < op.peer.size(); ++i) {
        if (op.sbase[i] == 4) a = std::max(a, op.soff[i] + op.sbytes[i]);
        if (op.rbase[i] == 5) b = std::max(b, op.roff[i] + op.rbytes[i]);
        sa += op.sbytes[i];   // host staging lays every peer's message side by side
        sb += op.rbytes[i];
      }
      if (op.type == 1 && op.bbase == 4) a = std::max(a, op.bytes);
      ss = std::max(ss, a);
      rs = std::max(rs, b);
      hs = std::max(hs, std::max(sa, op.type == 1 ? op.bytes : 0));
      hr = std::max(hr, std::max(sb, op.type == 1 ? op.bytes : 0));
    }
    h->stage_bytes_s = ss;
    h->stage_bytes_r = rs;
    HIPCHK(h->stage_s.alloc((size_t)(ss + 7) / 8 + 1));
    HIPCHK(h->stage_r.alloc((size_t)(rs + 7) / 8 + 1));
    if (!h->tr.device_memory) {
      HIPCHK(hipHostMalloc((void**)&h->hstage_s, (size_t)std::max<int64_t>(hs, 8), 0));
      HIPCHK(hipHostMalloc((void**)&h->hstage_r, (size_t)std::max<int64_t>(hr, 8), 0));
    }
    char* base[10] = {(char*)h->store.p, (char*)h->scratch.p, (char*)h->vbuf.p, (char*)h->wrk.p,
                      (char*)h->stage_s.p, (char*)h->stage_r.p, (char*)h->bcbuf.p, (char*)h->tinv.p,
                      (char*)h->swaps.p, (char*)h->rowperm.p};
    std::vector<SegDesc> d;
    for (CommOp& op : h->comm) {
      auto emit = [&](const std::vector<HSeg>& v, int64_t& at) {
        at = (int64_t)d.size();
        for (const HSeg& g : v)
          d.push_back(SegDesc{(uint64_t)(base[g.sb] + g.so), (uint64_t)(base[g.db] + g.dof), g.bytes / 4});
      };
      emit(op.pack, op.pack0);
      emit(op.unpack, op.unpack0);
    }
    HIPCHK(h->segdesc.upload(d.data(), d.size(), st));
  }
  HIPCHK(hipStreamSynchronize(st));
  return SMLU_OK;
}

static int setup_device(smlu_handle* h) {
  Plan& P = h->plan;
  HIPCHK(hipSetDevice(h->device));
  // one high-priority stream per handle (the schedule is one stream-ordered sequence)
  int prio_lo = 0, prio_hi = 0;
  HIPCHK(hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi));
  if (!h->stream) HIPCHK(hipStreamCreateWithPriority(&h->stream, hipStreamNonBlocking, prio_hi));
  hipStream_t st = h->stream;
  // this rank's layout: the plan's own on one GPU; ordinary fronts + owned column blocks of
  // the shared fronts on a partitioned handle
  if (h->nranks > 1) {
    rank_layout(P, h->rank, h->lay);
  } else {
    RankLayout& Y = h->lay;
    Y = RankLayout();
    Y.Loff = P.Loff;
    Y.Uoff = P.Uoff;
    Y.Foff = P.Foff;
    Y.recv_off.assign(P.nsup, -1);
    Y.recv_size.assign(P.nsup, 0);
    Y.store_size = P.factor_size;
    Y.scratch_size = P.scratch_size;
  }
  HIPCHK(h->A.alloc((size_t)std::max<int64_t>(P.nnzA, 1)));
  HIPCHK(h->Rs.alloc((size_t)P.n));
  // k_urows reads up to 64 columns and 16 rows past a block (values discarded): pad the store
  int64_t maxM = 1;
  for (int64_t s = 0; s < P.nsup; ++s) maxM = std::max<int64_t>(maxM, P.M(s));
  HIPCHK(h->store.alloc((size_t)(std::max<int64_t>(h->lay.store_size, 1) + 64 * maxM + 4096)));
  HIPCHK(h->scratch.alloc((size_t)std::max<int64_t>(h->lay.scratch_size, 1)));
  if (h->nranks > 1) {   // received pivot block + tile inverses + swap lists + rowperm
    int64_t bc = 1;
    for (int64_t s = 0; s < P.nsup; ++s)
      if (P.dist(s) && std::binary_search(P.group[s].begin(), P.group[s].end(), h->rank))
        bc = std::max<int64_t>(bc, P.M(s) * P.dob + (P.dob / 64) * 8192 + (P.dob / 64) * kSwapStride / 2 + P.dob / 2 + 64);
    HIPCHK(h->bcbuf.alloc((size_t)bc));
    HIPCHK(h->d_red.alloc(8));
  }
  HIPCHK(h->wrk.alloc((size_t)P.n));
  HIPCHK(h->wrk2.alloc((size_t)P.n));
  HIPCHK(h->growth.alloc(1));
  HIPCHK(h->Arowptr.upload(P.Arowptr.data(), P.Arowptr.size(), st));
  HIPCHK(h->Arow_ent.upload(P.Arow_ent.data(), P.Arow_ent.size(), st));
  HIPCHK(h->Arow.upload(P.Arow.data(), P.Arow.size(), st));
  HIPCHK(h->p0.upload(P.p0.data(), P.p0.size(), st));
  HIPCHK(h->q.upload(P.q.data(), P.q.size(), st));
  HIPCHK(h->rows.upload(P.s_rows.data(), P.s_rows.size(), st));
  HIPCHK(h->relmap.upload(P.relmap.data(), P.relmap.size(), st));
  HIPCHK(h->chlist.upload(P.ch_list.data(), P.ch_list.size(), st));
  std::vector<int64_t> pf(P.n);
  for (int64_t s = 0; s < P.nsup; ++s)
    for (int64_t j = P.s_first[s]; j < P.s_first[s + 1]; ++j) pf[j] = P.s_first[s];
  HIPCHK(h->posfirst.upload(pf.data(), pf.size(), st));
  HIPCHK(h->rowperm.alloc((size_t)P.n));
  {
    std::vector<int32_t> id(P.n);
    for (int64_t j = 0; j < P.n; ++j) id[j] = (int32_t)(j - pf[j]);
    HIPCHK(h->rowperm0.upload(id.data(), id.size(), st));
  }
  const int64_t nnodes = P.nsup + (int64_t)h->lay.blocks.size();
  HIPCHK(h->info.alloc((size_t)std::max<int64_t>(nnodes, 1)));
  HIPCHK(init_kernel_attributes());
  if (!h->rb.p) HIPCHK(h->rb.alloc(16));
  return build_schedule(h);
}

// --- event-timed execution (profile mode) ---
struct Timer {
  smlu_handle* h;
  size_t used = 0;
  explicit Timer(smlu_handle* hh) : h(hh) {}
  hipStream_t st = nullptr;
  hipError_t begin(int kind, hipEvent_t* stop, hipStream_t s) {
    st = s;
    if (!h->opts.profile) { *stop = nullptr; return hipSuccess; }
    if (used == h->ev_pool.size()) {
      hipEvent_t a, b;
      hipError_t e = hipEventCreate(&a);
      if (e != hipSuccess) return e;
      e = hipEventCreate(&b);
      if (e != hipSuccess) return e;
      h->ev_pool.push_back({a, b});
      h->ev_kind.push_back(kind);
    }
    h->ev_kind[used] = kind;
    *stop = h->ev_pool[used].second;
    hipError_t e = hipEventRecord(h->ev_pool[used].first, st);
    ++used;
    return e;
  }
  hipError_t end(hipEvent_t stop) { return stop ? hipEventRecord(stop, st) : hipSuccess; }
  void collect() {
    for (size_t i = 0; i < used; ++i) {
      float ms = 0;
      if (hipEventElapsedTime(&ms, h->ev_pool[i].first, h->ev_pool[i].second) == hipSuccess)
        h->kind_ms[h->ev_kind[i]] += ms;
      else
        (void)hipGetLastError();   // a pair not recorded this time: no sticky error for the caller's next API call
    }
  }
};

static hipError_t run_launch(smlu_handle* h, const Launch& L, double diag_tol, double piv_tol) {
  hipStream_t st = h->stream;
  switch (L.kind) {
    case K_MEMSET_STORE:
      return hipMemsetAsync(h->store.p + L.off, 0, (size_t)L.cnt * sizeof(double), st);
    case K_MEMSET_SCRATCH:
      return hipMemsetAsync(h->scratch.p + L.off, 0, (size_t)L.cnt * sizeof(double), st);
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
  for (size_t li = lo; li < hi; ++li) {
    const Launch& L = h->fac[li];
    hipEvent_t stop;
    HIPCHK(tm.begin(L.kind, &stop, st));
    hipError_t e = run_launch(h, L, diag_tol, piv_tol);
    if (e == hipSuccess && dbg) e = hipStreamSynchronize(st);
    if (e != hipSuccess) {
      char buf[256];
      std::snprintf(buf, sizeof buf, "HIP error '%s' in launch kind=%d step=%d off=%lld cnt=%lld nwg=%lld aux=%lld aux2=%lld",
                    hipGetErrorString(e), L.kind, L.step, (long long)L.off, (long long)L.cnt,
                    (long long)L.nwg, (long long)L.aux, (long long)L.aux2);
      return fail(h, SMLU_ERR_HIP, buf);
    }
    HIPCHK(tm.end(stop));
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
static int read_status(smlu_handle* h, const int32_t* info, int64_t nnodes, const int32_t* words, int nwords,
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
  int rs = read_status(h, h->info.p, h->nnodes, reinterpret_cast<const int32_t*>(h->growth.p), 2, rec);
  if (rs != SMLU_OK) return rs;
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
static int exec_comm(smlu_handle* h, int id) {
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

// Schedule-dependent device buffers and graphs (rebuilt when the pivoting mode changes).
static void release_schedule(smlu_handle* h) {
  h->release_graphs();
  h->sn.free();
  h->ilist.free();
  h->xtasks.free();
  h->aents.free();
  h->ftiles.free();
  h->gptr.free();
  h->gent.free();
  h->ssync.free();
  h->stick.free();
  h->sxh.free();
  h->gtasks.free();
  h->stasks.free();
  h->urtasks.free();
  h->xcols.free();
  h->swaps.free();
  h->vbuf.free();
  h->vbufm.free();
  h->tinv.free();
  h->stage_s.free();
  h->stage_r.free();
  h->segdesc.free();
  if (h->hstage_s) (void)hipHostFree(h->hstage_s);
  if (h->hstage_r) (void)hipHostFree(h->hstage_r);
  h->hstage_s = h->hstage_r = nullptr;
}

static int rebuild_schedule(smlu_handle* h) {
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(hipStreamSynchronize(h->stream));
  release_schedule(h);
  return build_schedule(h);
}

static bool has_tile_fronts(const smlu_handle* h) {
  for (const SNode& r : h->hsn)
    if (r.mode == 2) return true;
  return false;
}

// One numeric factorization with the re-pivoting fallback (UMFPACK re-pivots in
// every lu!, src/SharedMemSparseLU.jl:247): the diagonal-tile pivoting of large fronts only
// searches the 64x64 diagonal tile.  When it meets a zero pivot (the matrix may still be
// nonsingular: a zero diagonal block) or accepts weak pivots, the same values are factored
// again with full-candidate pivoting (every fully-summed row of the front) in every blocked
// front, and the handle keeps that mode until a refactor's host values are diagonally dominant
// again.  A given (p, q) is never re-pivoted.
static int run_factor(smlu_handle* h) {
  int rc = run_factor_once(h);
  if (rc < 0) return rc;
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

// One solve launch for rh.n right-hand sides (x columns at w + r*rh.ldx, front vectors at
// v + r*rh.ldv); the multi-GPU kinds (K_BWDU12C, K_VCOPY) are single-vector only.
static hipError_t run_solve_launch(smlu_handle* h, const Launch& L, double* w, double* v, Rhs rh) {
  hipStream_t st = h->stream;
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
  constexpr int sweep_max_rhs = 1;   // batches run the per-block schedule (the NR-wide sweep slots measured slower)
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
  auto run_seq = [&](const std::vector<Launch>& seq, const std::vector<size_t>& seg, const std::vector<int>& cm) {
    for (size_t k = 0; k < seg.size(); ++k) {
      if (k > 0) {
        int rc = exec_comm(h, cm[k - 1]);
        if (rc != SMLU_OK) return rc;
      }
      const size_t hi = k + 1 < seg.size() ? seg[k + 1] : seq.size();
      for (size_t i = seg[k]; i < hi; ++i) HIPCHK(run_solve_launch(h, seq[i], w, v, rh));
    }
    return (int)SMLU_OK;
  };
  auto sweeps = [&](bool steps) {   // steps: the per-block sequences instead of the sweeps
    if (mode != 2) {
      int rc = steps ? run_seq(h->fwdm, h->fwdm_seg, h->fwd_comm) : run_seq(h->fwd, h->fwd_seg, h->fwd_comm);
      if (rc != SMLU_OK) return rc;
    }
    if (mode != 1) {
      int rc = steps ? run_seq(h->bwdm, h->bwdm_seg, h->bwd_comm) : run_seq(h->bwd, h->bwd_seg, h->bwd_comm);
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

static bool valid_opts(const smlu_opts* o) { return o && (o->index_base == 0 || o->index_base == 1); }

// Diagonal dominance of A by columns or by rows (|a_jj| >= sum of the other |a_ij|, a_jj != 0).
template <class RI>
static bool diagonally_dominant(int64_t n, const int64_t* colptr, const RI* rowval, const double* a,
                                int64_t base) {
  std::vector<double> rdiag(n, 0.0), roff(n, 0.0);
  bool col_dom = true;
  for (int64_t j = 0; j < n; ++j) {
    double d = 0.0, off = 0.0;
    for (int64_t e = colptr[j] - base; e < colptr[j + 1] - base; ++e) {
      const int64_t i = rowval[e] - base;
      const double v = std::fabs(a[e]);
      if (i == j) { d += v; rdiag[i] += v; }
      else { off += v; roff[i] += v; }
    }
    if (!(d > 0.0 && d >= off)) col_dom = false;
  }
  if (col_dom) return true;
  for (int64_t i = 0; i < n; ++i)
    if (!(rdiag[i] > 0.0 && rdiag[i] >= roff[i])) return false;
  return true;
}

// Row transversal for a zero-free diagonal (ordering.cpp: zero_free_diagonal), computed only
// when A has a structurally or exactly zero diagonal entry; empty = not needed / not possible.
static std::vector<int64_t> diagonal_match(int64_t n, const int64_t* colptr, const int64_t* rowval,
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

static int create_impl(int64_t n, const int64_t* colptr, const int64_t* rowval, const double* nzval,
                       const int64_t* p, const int64_t* q, const double* Rs, const smlu_opts* opts,
                       smlu_handle** out, int rank = 0, int nranks = 1, const smlu_transport* tr = nullptr,
                       RcclState* rccl = nullptr, const std::vector<int64_t>* preorder = nullptr) {
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
extern "C" {

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

static int ensure_residual(smlu_handle* h);

// Pivoting mode per refactor: dominant values take the diagonal-tile path for
// the mid-size fronts; a handle left in full-candidate mode by a re-pivoting refactor returns to
// the fast schedule once the values are dominant again.  The ranks of a partitioned handle agree
// on the decision (any rank seeing non-dominant values makes it non-dominant for all): a rebuild
// on only some ranks would split the collective schedule.
static int apply_dominance(smlu_handle* h, bool dom) {
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
  return changed ? rebuild_schedule(h) : SMLU_OK;
}

// The same dominance test on values already in HBM (k_dominance: one thread per column and row,
// the host's summation order), for device-only callers.
static int device_dominant(smlu_handle* h, bool* dom) {
  const Plan& P = h->plan;
  hipStream_t st = h->stream;
  if (!h->Acolp.p) {
    HIPCHK(h->Acolp.upload(P.Acolptr.data(), P.Acolptr.size(), st));
    HIPCHK(h->domflag.alloc(2));
  }
  int rc = ensure_residual(h);   // the column of every A entry
  if (rc != SMLU_OK) return rc;
  HIPCHK(launch_dominance(st, P.n, h->Acolp.p, h->Arow.p, h->Arowptr.p, h->Arow_ent.p, h->Acol.p, h->A.p,
                          h->domflag.p));
  long long rec[16];
  rc = read_status(h, nullptr, 0, h->domflag.p, 2, rec);
  if (rc != SMLU_OK) return rc;
  *dom = (rec[6] & 0xffffffffll) != 0 || (rec[6] >> 32) != 0;
  return SMLU_OK;
}

// lu! on the values already in h->A: the pivoting mode re-decided on the device, then the
// factorization (with the re-pivoting fallback).
static int refactor_resident(smlu_handle* h) {
  if (!h->plan.given_order && !h->plan.matched) {
    bool dom = false;
    int rc = device_dominant(h, &dom);
    if (rc == SMLU_OK) rc = apply_dominance(h, dom);
    if (rc != SMLU_OK) return rc;
  }
  return run_factor(h);
}

int smlu_refactor(smlu_handle* h, const double* nzval) {
  if (!h || !nzval) return fail(h, SMLU_ERR_ARG, "NULL argument");
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(hipMemcpyAsync(h->A.p, nzval, sizeof(double) * h->plan.nnzA, hipMemcpyHostToDevice, h->stream));
  if (!h->plan.given_order && !h->plan.matched) {   // pivoting mode per refactor: re-check dominance
    const Plan& P = h->plan;
    int rc = apply_dominance(h, diagonally_dominant(P.n, P.Acolptr.data(), P.Arow.data(), nzval, 0));
    if (rc != SMLU_OK) return rc;
  }
  return run_factor(h);   // collective on a partitioned handle
}

// Device entry points read caller memory (values, right-hand sides) on the handle's own stream:
// order that stream after the work the caller has enqueued on its stream so far (an event, no
// host wait).  Outputs are complete when an entry point returns (it synchronises its stream).
static hipError_t after_caller(smlu_handle* h) {
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

static int refactor_csc_impl(smlu_handle* h, int64_t n, const int64_t* colptr, const int64_t* rowval,
                             const double* nzval, const std::vector<int64_t>* preorder);

int smlu_refactor_csc(smlu_handle* h, int64_t n, const int64_t* colptr, const int64_t* rowval,
                      const double* nzval) {
  if (!h || !colptr || !rowval || !nzval) return fail(h, SMLU_ERR_ARG, "NULL argument");
  if (h->zc) return fail(h, SMLU_ERR_ARG, "complex handle: use smlu_refactor_csc_z");
  return refactor_csc_impl(h, n, colptr, rowval, nzval, nullptr);
}

}  // extern "C"

static int refactor_csc_impl(smlu_handle* h, int64_t n, const int64_t* colptr, const int64_t* rowval,
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

extern "C" {

}  // extern "C"

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

extern "C" {

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

}  // extern "C"

extern "C" {

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
static int ensure_residual(smlu_handle* h) {
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

// ---- factor export ------------------------------------------------------------------
struct Exported {
  std::vector<int64_t> Lp, Li, Up, Ui, p, q;
  std::vector<double> Lx, Ux;
};

// Exact structural pattern of L and U for B = (Rs.*A)[p, q] with the pivot sequence fixed
// (X.p, X.q already set): column k of L+U is the reach of pattern(B(:,k)) in the graph of
// L(:, 0:k-1) (Gilbert-Peierls symbolic step; the diagonal of U is always stored).  Values
// come from the fronts: L(i,k) from the L panel of k's front (own rows in their final
// position, update rows looked up by their pre-interchange position), U(i,k) from the
// diagonal block or U12 of i's front.  Every structural entry lies in the front
// (pattern(A+A') contains it), otherwise the export fails.
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

static int export_factors(smlu_handle* h, Exported& X, bool values) {
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
      const bool mfma = L.aux == 130 || L.aux == 131 || L.aux == 135;
      if (v == "mfma128" && gemm && mfma) ++c;
      else if (v == "mfma128_trsm" && trsm && mfma) ++c;
      else if (v == "valu128" && gemm && L.aux == 128) ++c;
      else if (v == "k64" && gemm && L.aux == 65) ++c;
      else if (v == "k64_trsm" && trsm && L.aux == 65) ++c;
      else if (v == "valu64" && gemm && L.aux == 64) ++c;
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

const char* smlu_version(void) { return "smlu 0.1.0 (gfx950, fp64, multifrontal)"; }

}  // extern "C"
