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
#include <cstdint>
#include <string>
#include <vector>

namespace smlu {

struct PlanOptions {
  int ordering = 0;          // SMLU_ORDER_*
  int64_t grid[3] = {0, 0, 0};
  int relax = 1;
  int64_t leaf_size = 64;
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

  // ---- multi-GPU partition (compute_owners) ----
  // owner[s] = rank that factors front s.  Proportional mapping of the assembly tree: a
  // subtree whose rank set has one member is owned by it entirely; a front above that keeps
  // the first rank of its set.  Exchange points are the levels of fronts with a child owned
  // by another rank (the child's update block crosses GPUs right before that level).
  int nparts = 1;
  std::vector<int32_t> owner;
  std::vector<int32_t> xlevels;               // sorted exchange-point levels
  std::vector<double> front_flops;            // per front (same formula as `flops`)
  void compute_owners(int nparts);

  std::string build(int64_t n, const int64_t* colptr, const int64_t* rowval, int index_base,
                    const PlanOptions& opt, const int64_t* pgiven = nullptr,
                    const int64_t* qgiven = nullptr, const int64_t* rowmatch = nullptr);

  int64_t ns(int64_t s) const { return s_first[s + 1] - s_first[s]; }
  int64_t nu(int64_t s) const { return s_rowptr[s + 1] - s_rowptr[s]; }
  int64_t M(int64_t s) const { return ns(s) + nu(s); }
  // local index of global (new) position g inside front s, or -1
  int64_t local_index(int64_t s, int64_t g) const;
};

}  // namespace smlu
