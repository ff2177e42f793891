// handle.hpp — internal to libsmlu.so: the handle, the launch records of its static schedule,
// device buffers, the built-in RCCL transport and the host entry points shared by the units
//   schedule.cpp  (schedule construction, device set-up)   factor.cpp  (refactorization)
//   solve.cpp     (solves, refinement, chunked layout)     export.cpp  (factor export, pattern hand-over)
//   complex.cpp   (ComplexF64 handles)                     dist.cpp    (RCCL, partitioned handles)
//   smlu.cpp      (create / destroy / stats / plan API)
#pragma once
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

namespace smlu {

constexpr int kSmallM = 128;     // fronts up to this order are factored whole in LDS
constexpr int kFullPivNs = 512;  // blocked fronts up to this many pivots search all fully-summed rows
constexpr int kNbFull = 32;
constexpr int kNbTile = 64;
constexpr int kSwapStride = 1 + 2 * 64;
constexpr int kOBDefault = 384;   // outer block of the two-level blocked front factorization (256/384/512 within 1 %; 384 best)

extern thread_local std::string g_last_error;

enum Kind : int {
  K_EXTADD, K_FRONT_LDS, K_PANEL, K_TRSMU, K_TRSML,
  K_GEMM, K_FWD, K_BWD, K_FWDG, K_TRIF, K_BWDU, K_TRIB, K_GEMM22, K_LASWP, K_STEPTRSM, K_GEMMU,
  K_GEMMO, K_TRIINV, K_BWDU12C, K_VCOPY, K_FWDT, K_BWDT, K_SWEEPF, K_SWEEPB, K_UROWS, K_FWDP, K_NKIND
};
inline const char* const kKindName[] = {"assemble", "small", "panel",
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
  // solves (one GPU): consecutive launches with the same grp > 0 are one level's fronts; in batched
  // solves (the per-block schedule) the side ones (small and tiny fronts) run on the handle's side
  // stream next to the large fronts' chain
  int grp = 0;
  bool side = false;
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

RcclApi* rccl_api();

struct RcclState {
  ncclComm_t comm = nullptr;
  int rank = 0;
  int comm_count = 0;             // ranks in the communicator (ncclCommCount after init)
  hipStream_t stream = nullptr;   // the handle's stream (allreduce)
  double* dbuf = nullptr;         // device scratch for the allreduce
};

// point-to-point batch over xGMI: sends and receives of all peers in one group
int rccl_exchange(void* ctx, int32_t npeer, const int32_t* peer, void* const* sbuf, const int64_t* sbytes,
                  void* const* rbuf, const int64_t* rbytes, void* stream);
int rccl_bcast(void* ctx, void* buf, int64_t bytes, int32_t root, int32_t gsize, const int32_t* group, void* stream);
int rccl_allreduce_max(void* ctx, double* buf, int32_t count);

}  // namespace smlu

struct smlu_plan {
  Plan plan;
};

struct smlu_handle {
  smlu_opts opts{};
  Plan plan;
  int device = 0;
  hipStream_t stream = nullptr;
  // second stream of the factor sequence: the small-front size classes of one level run on two
  // streams (fork / join by events, captured into the same graph as parallel branches)
  hipStream_t side = nullptr;
  hipEvent_t fork_ev = nullptr, join_ev = nullptr;
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
  bool host_only = false;      // schedule built without a device (smlu_plan_rank_schedule)
  double host_bytes[5] = {0};  // ... and the bytes it would allocate (build_schedule_host)
  int ob = kOBDefault;        // outer block width (SMLU_OB overrides; multiple of 64)
  int64_t t128_min = 512;     // 128x128 GEMM tiles when a launch has at least this many
  bool small_k = true;        // k <= 64 launches use k_gemm_k64 (SMLU_SMALLK=0: off)
  bool dominant = false;      // A diagonally dominant (by rows or columns): last host values seen
  int pivmode = 0;            // 0: diagonal-tile pivoting for large (and, if dominant, mid-size)
                              //    fronts; 1: full-candidate pivoting in every blocked front (the
                              //    re-pivoting refactor after a zero or weak tile pivot)
  int64_t repivots = 0;       // re-pivoting refactors run so far
  int64_t mode_refactors = 0; // factorizations repeated because the values called for another pivoting mode
  long long dom_words = 0;    // dominance flags (columns | rows << 32) in the last factorization's record
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
    if (fork_ev) (void)hipEventDestroy(fork_ev);
    if (join_ev) (void)hipEventDestroy(join_ev);
    fork_ev = join_ev = nullptr;
    if (side) (void)hipStreamDestroy(side);
    side = nullptr;
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

inline int fail(smlu_handle* h, int code, const std::string& msg) {
  if (h) h->err = msg;
  g_last_error = msg;
  return code;
}

inline PlanOptions plan_opts(const smlu_opts& o) {
  PlanOptions p;
  p.ordering = o.ordering;
  for (int i = 0; i < 3; ++i) p.grid[i] = o.grid[i];
  p.relax = o.relax;
  p.leaf_size = o.leaf_size > 0 ? o.leaf_size : 64;
  return p;
}

inline bool valid_opts(const smlu_opts* o) { return o && (o->index_base == 0 || o->index_base == 1); }

// Diagonal dominance of A by columns or by rows (|a_jj| >= sum of the other |a_ij|, a_jj != 0).
template <class RI>
bool diagonally_dominant(int64_t n, const int64_t* colptr, const RI* rowval, const double* a,
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

// ---- entry points shared between the units (defined in the unit named) ----
int create_impl(int64_t n, const int64_t* colptr, const int64_t* rowval, const double* nzval, const int64_t* p,
                const int64_t* q, const double* Rs, const smlu_opts* opts, smlu_handle** out, int rank = 0,
                int nranks = 1, const smlu_transport* tr = nullptr, RcclState* rccl = nullptr,
                const std::vector<int64_t>* preorder = nullptr);   // smlu.cpp
std::vector<int64_t> diagonal_match(int64_t n, const int64_t* colptr, const int64_t* rowval, const double* a,
                                    int64_t base);   // smlu.cpp
int setup_device(smlu_handle* h);                        // schedule.cpp
int build_schedule_host(smlu_handle* h);
int rebuild_schedule(smlu_handle* h);
bool has_tile_fronts(const smlu_handle* h);
int run_factor(smlu_handle* h, bool redecide = false);   // factor.cpp
int read_status(smlu_handle* h, const int32_t* info, int64_t nnodes, const int32_t* words, int nwords,
                long long out[16]);
hipError_t after_caller(smlu_handle* h);
int refactor_resident(smlu_handle* h);
int refactor_csc_impl(smlu_handle* h, int64_t n, const int64_t* colptr, const int64_t* rowval,
                      const double* nzval, const std::vector<int64_t>* preorder);
int exec_comm(smlu_handle* h, int id);                   // dist.cpp
int ensure_residual(smlu_handle* h);                     // solve.cpp


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
int export_factors(smlu_handle* h, Exported& X, bool values);   // export.cpp
