// plan.hpp — host symbolic analysis for the MI355X sparse LU (smlu).
//
// The reference (SharedMemSparseLU.jl) delegates ordering + symbolic + numeric LU to UMFPACK
// (`lu(A)`, src/SharedMemSparseLU.jl:74; `lu!(F.lu_object, A)`, :247).  Here the symbolic
// part stays on the host, as the north star asks, and is designed for a level-scheduled
// multifrontal numeric phase on the GPU:
//   ordering (geometric / graph nested dissection) -> elimination tree of A+A' -> postorder
//   -> column counts (Gilbert-Ng-Peyton) -> supernodes -> relaxed amalgamation
//   -> per-supernode update-row structure -> levels (height in the assembly tree)
//   -> HBM layout of factor panels and the scratch arena for update (F22) blocks
//   -> map of every A entry to its slot in a front.
#pragma once
#include <algorithm>
#include <cstdint>
#include <string>
#include <vector>

namespace smlu {

// Tuning / test knobs of the library, read from the environment by tune() (tune.cpp, the only
// place libsmlu reads it; documented in include/smlu.h).  Anything not listed here is not a knob.
struct Tune {
  int ob = 0;                 // SMLU_OB: outer block width (multiple of 64; 0 = the default 384)
  int64_t t128_min = 512;     // SMLU_T128MIN: 128x128 MFMA tiles from this many output tiles per launch
  bool small_k = true;        // SMLU_SMALLK=0: no one-shot k <= 64 GEMM tile
  int64_t fullpiv_ns = -1;    // SMLU_FULLPIV_NS: largest ns with full-candidate pivoting (-1 = default rule)
  int sweep_spin = 1 << 22;   // SMLU_SWEEP_SPIN: polls before a sync-free solve wait gives up (0: at once)
  bool solve_steps = false;   // SMLU_SOLVE_STEPS=1: per-block solve launches instead of the sweeps
  bool no_graph = false;      // SMLU_NO_GRAPH: eager launches, no captured graphs
  bool debug_sync = false;    // SMLU_DEBUG_SYNC: synchronise after every launch (error localisation)
  bool no_repivot = false;    // SMLU_NO_REPIVOT: no re-pivoting refactor after weak tile pivots
  int host_threads = 0;       // OMP_NUM_THREADS: cap on the analysis threads (0 = not set)
};
Tune tune();


struct PlanOptions {
  int ordering = 0;          // SMLU_ORDER_*
  int64_t grid[3] = {0, 0, 0};
  int relax = 1;
  int64_t leaf_size = 64;
  // Column order to use instead of computing one (new -> old, 0-based; empty = compute).
  // Pivoting stays on, unlike a given (p, q).  Used by the ComplexF64 path: the order is
  // computed on the complex pattern and expanded to the real-equivalent 2x2 blocks.
  std::vector<int64_t> preorder;
};

// Symmetric adjacency (A + A'), no diagonal, deduplicated, CSR.
struct Graph {
  int64_t n = 0;
  std::vector<int64_t> ptr;
  std::vector<int32_t> adj;
};

Graph build_sym_graph(int64_t n, const int64_t* colptr, const int32_t* rowval);
// Orderings return perm (new -> old).
std::vector<int64_t> order_geometric_nd(int64_t nx, int64_t ny, int64_t nz, int64_t leaf);
std::vector<int64_t> order_graph_nd(const Graph& g, int64_t leaf);
std::vector<int64_t> order_amd(const Graph& g);   // approximate minimum degree (amd.cpp)
// The ordering Plan::build would compute for the pattern (0-based CSC) under `opt`
// (natural / geometric ND / AMD / graph ND); empty with `err` set on a bad option.
std::vector<int64_t> compute_order(int64_t n, const int64_t* colptr, const int32_t* rowval,
                                   const PlanOptions& opt, std::string& err);
std::vector<int64_t> zero_free_diagonal(int64_t n, const int64_t* colptr, const int32_t* rowval,
                                        const double* a);

struct Plan {
  // ---- input pattern (0-based copy) ----
  int64_t n = 0, nnzA = 0;
  std::vector<int64_t> Acolptr;
  std::vector<int32_t> Arow;
  bool sym_pattern = false;       // pattern(A) == pattern(A'): the plan's structure is exact

  // ---- orderings: new -> old and inverses ----
  std::vector<int64_t> q, qinv;   // columns
  std::vector<int64_t> p0, p0inv; // rows (== q unless given)
  bool given_order = false;
  bool matched = false;           // rows pre-permuted by a zero-free-diagonal transversal

  // ---- exact (pre-relaxation) supernodes: structure of L column j in t=col2t[j] is
  //      {j..last(t)} U R_t  (R_t sorted, all > last(t)) ----
  int64_t ntsup = 0;
  std::vector<int64_t> t_first;               // ntsup+1
  std::vector<int64_t> t_rowptr;              // ntsup+1
  std::vector<int32_t> t_rows;
  std::vector<int32_t> col2t;

  // ---- relaxed supernodes (the fronts of the multifrontal factorization) ----
  int64_t nsup = 0;
  std::vector<int64_t> s_first;               // nsup+1
  std::vector<int64_t> s_parent;              // -1 = root
  std::vector<int64_t> s_rowptr;              // nsup+1 ; update rows R_s
  std::vector<int32_t> s_rows;
  std::vector<int32_t> col2s;
  std::vector<int32_t> s_level;
  std::vector<int64_t> ch_ptr;                // children of s, in postorder
  std::vector<int32_t> ch_list;
  std::vector<int32_t> child_rank;            // rank of s among its parent's children
  std::vector<int32_t> relmap;                // per update row of s: local index in parent front
  int nlevels = 0;
  std::vector<int64_t> lev_ptr;               // nlevels+1
  std::vector<int32_t> lev_sup;               // supernodes ordered by level

  // ---- HBM layout (units: doubles) ----
  // factor store: per s, L panel (M x ns, ld M) at Loff[s], U12 (ns x nu, ld ns) at Uoff[s];
  // ordered by level so that a level's panels are one contiguous range [lev_foff[l], lev_foff[l+1]).
  std::vector<int64_t> Loff, Uoff;
  std::vector<int64_t> lev_foff;              // nlevels+1
  int64_t factor_size = 0;
  // scratch arena for F22 (nu x nu, ld nu): one block per level, first-fit by liveness.
  std::vector<int64_t> Foff;
  std::vector<int64_t> lev_soff, lev_ssize;   // per level block
  int64_t scratch_size = 0;

  // ---- A entry -> front slot ----
  // dest >= 0: factor store offset;  dest < 0: scratch offset (-1 - dest)
  std::vector<int64_t> Adest;
  std::vector<int32_t> A_s, A_li, A_lj;       // front, local row, local column of each entry
  std::vector<int64_t> Alev_ptr;              // nlevels+1
  std::vector<int32_t> Alev_ent;              // A entry ids grouped by level, sorted by dest
  // row-scaling support: A entries grouped by row (CSR order of A)
  std::vector<int64_t> Arowptr;               // n+1
  std::vector<int32_t> Arow_ent;              // entry ids

  // ---- statistics ----
  double nnzL = 0, nnzU = 0;   // exact structural counts (L incl. unit diagonal)
  double upd = 0;              // sum_k |L_k| |U_k| (exact structure)
  double flops = 0;            // dense flops actually executed over relaxed fronts
  double stored = 0;           // doubles stored in factor panels
  int64_t front_max = 0, ns_max = 0, nu_max = 0;
  double analysis_ms = 0;
  // analysis phases (ms): input, graph, ordering, etree, column counts, row structures, relax,
  // levels / relmap, layout, A map (10, 11: the A map's entry pass and its level sort)
  double phase_ms[12] = {0};

  // ---- multi-GPU partition (compute_owners) ----
  // Subtrees of the assembly tree are bin-packed onto ranks (each factored with no
  // communication).  A front above them ("top" front) is shared by the group of ranks that own
  // its subtrees: its columns are split into blocks of `dob` columns dealt round-robin over the
  // group (pivot blocks first, then the update-column blocks), a 1D block-cyclic column
  // partition of the dense front.  A front whose group has one rank is an ordinary front of
  // that rank.
  int nparts = 1;
  int64_t dob = 384;                          // column block of the distributed fronts
  std::vector<int32_t> owner;                 // rank of an ordinary front, -1 for a distributed one
  std::vector<std::vector<int32_t>> group;    // per front: sorted ranks (size 1: ordinary)
  std::vector<double> front_flops;            // per front (same formula as `flops`)
  void compute_owners(int nparts, int64_t block = 384);
  bool dist(int64_t s) const { return !group.empty() && group[s].size() > 1; }
  int64_t npblk(int64_t s) const { return (ns(s) + dob - 1) / dob; }
  int64_t nublk(int64_t s) const { return (nu(s) + dob - 1) / dob; }
  // owner of column block b of front s (b < npblk: pivot columns [b*dob, ..), else update
  // columns [ns + (b - npblk)*dob, ..))
  int32_t blk_owner(int64_t s, int64_t b) const { return group[s][b % group[s].size()]; }
  int64_t blk_c0(int64_t s, int64_t b) const {
    const int64_t np = npblk(s);
    return b < np ? b * dob : ns(s) + (b - np) * dob;
  }
  int64_t blk_c1(int64_t s, int64_t b) const {
    const int64_t np = npblk(s);
    return b < np ? std::min(ns(s), (b + 1) * dob) : std::min(M(s), ns(s) + (b - np + 1) * dob);
  }
  int32_t col_owner(int64_t s, int64_t c) const {
    if (!dist(s)) return owner[s];
    return c < ns(s) ? blk_owner(s, c / dob) : blk_owner(s, npblk(s) + (c - ns(s)) / dob);
  }

  std::string build(int64_t n, const int64_t* colptr, const int64_t* rowval, int index_base,
                    const PlanOptions& opt, const int64_t* pgiven = nullptr,
                    const int64_t* qgiven = nullptr, const int64_t* rowmatch = nullptr);

  int64_t ns(int64_t s) const { return s_first[s + 1] - s_first[s]; }
  int64_t nu(int64_t s) const { return s_rowptr[s + 1] - s_rowptr[s]; }
  int64_t M(int64_t s) const { return ns(s) + nu(s); }
  // local index of global (new) position g inside front s, or -1
  int64_t local_index(int64_t s, int64_t g) const;
};

// Device memory layout of one rank (units: doubles).  Ordinary fronts of the rank: L panel and
// U12 in the factor store, F22 in the scratch arena (first-fit by liveness, live until the
// parent's level).  Distributed fronts: per owned column block, pivot blocks as M x w
// full-height L columns in the store; update blocks as their U12 rows (ns x w) in the store
// and F22 rows (nu x w) in the scratch arena; plus a receive area per distributed front for
// the children's F22 columns arriving from other ranks (live at the front's level only).
struct RankLayout {
  int rank = 0;
  std::vector<int64_t> Loff, Uoff, Foff;      // ordinary fronts of this rank (-1 elsewhere)
  struct Blk {
    int32_t s;          // front
    int32_t b;          // block index (pivot blocks first)
    int64_t c0, c1;     // columns
    int64_t loff;       // pivot block: L columns (ld M); update block: U12 rows (ld ns)
    int64_t foff;       // update block: F22 rows (ld nu) in scratch, -1 otherwise
  };
  std::vector<Blk> blocks;                    // owned blocks of distributed fronts
  std::vector<int64_t> recv_off, recv_size;   // per front: receive area for child F22 columns
  int64_t store_size = 0, scratch_size = 0;
  int64_t stage_size = 0;                     // largest block broadcast (doubles)
};
void rank_layout(const Plan& P, int rank, RankLayout& out);
// Critical-path projection of the partitioned factorization (host model): per front, the
// flops of its work per rank at `tflops`, the block broadcasts and child F22 exchanges at
// `gbs` GB/s and `lat_us` per message; returns the projected time (s) and the one-GPU time.
double project_partition(const Plan& P, double tflops, double gbs, double lat_us, double* t1);

}  // namespace smlu
