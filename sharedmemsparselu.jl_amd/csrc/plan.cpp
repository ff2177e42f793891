// plan.cpp — host symbolic analysis (see plan.hpp for the pipeline).
//
// Parity notes against the reference:
//  * UMFPACK's contract F.L*F.U == (F.Rs .* A)[F.p, F.q] (src/SharedMemSparseLU.jl:305-316)
//    is kept: q is the column order built here, p = q composed with the row interchanges
//    chosen inside each front by the GPU (threshold partial pivoting, diagonal preference).
//  * The exact structural pattern of L (and U = its transpose pattern) is recorded from the
//    pre-relaxation supernodes so that exported factors carry the structural fill of
//    (Rs.*A)[p,q] and nothing else.
#include <algorithm>
#include <cstdlib>
#include <functional>
#include <map>
#include <chrono>
#include <cmath>
#include <cstring>
#include <numeric>
#include <stdexcept>
#include <thread>
#include <atomic>

#include "plan.hpp"

#include <cstdio>

namespace smlu {

int64_t Plan::local_index(int64_t s, int64_t g) const {
  int64_t f = s_first[s], l = s_first[s + 1];
  if (g >= f && g < l) return g - f;
  const int32_t* b = s_rows.data() + s_rowptr[s];
  const int32_t* e = s_rows.data() + s_rowptr[s + 1];
  const int32_t* it = std::lower_bound(b, e, (int32_t)g);
  if (it == e || *it != g) return -1;
  return (l - f) + (it - b);
}

namespace {

// Host threads for the analysis: the hardware threads, at most 32, and at most OMP_NUM_THREADS
// when that is set (the 256^3 plan is built on every rank of a node, each rank with its share).
int plan_threads() {
  static const int t = [] {
    int v = (int)std::min(32u, std::max(1u, std::thread::hardware_concurrency()));
    const int cap = tune().host_threads;
    return cap > 0 ? std::min(v, cap) : v;
  }();
  return t;
}

// f(lo, hi) over [0, n) in contiguous chunks on plan_threads() threads.
template <class F>
void parallel_for(int64_t n, F&& f, int64_t grain = 65536) {
  const int T = (int)std::min<int64_t>(plan_threads(), std::max<int64_t>(1, n / grain));
  if (T <= 1) { f((int64_t)0, n); return; }
  std::vector<std::thread> th;
  th.reserve(T - 1);
  for (int t = 1; t < T; ++t) th.emplace_back([&f, n, T, t] { f(n * t / T, n * (t + 1) / T); });
  f((int64_t)0, n / T);
  for (auto& x : th) x.join();
}

// std::sort of [b, e) in parallel chunks merged pairwise (same result as std::sort for a strict
// weak order whose equivalent elements are identical, e.g. distinct keys).
template <class It, class Cmp>
void parallel_sort(It b, It e, Cmp cmp) {
  const int64_t n = e - b;
  const int T = (int)std::min<int64_t>(plan_threads(), std::max<int64_t>(1, n / 262144));
  if (T <= 1) { std::sort(b, e, cmp); return; }
  std::vector<int64_t> cut(T + 1);
  for (int t = 0; t <= T; ++t) cut[t] = n * t / T;
  parallel_for(T, [&](int64_t lo, int64_t hi) {
    for (int64_t t = lo; t < hi; ++t) std::sort(b + cut[t], b + cut[t + 1], cmp);
  }, 1);
  for (int w = 1; w < T; w *= 2) {
    std::vector<std::thread> th;
    for (int t = 0; t + w < T; t += 2 * w) {
      const int64_t lo = cut[t], mid = cut[t + w], hi = cut[std::min(T, t + 2 * w)];
      th.emplace_back([=] { std::inplace_merge(b + lo, b + mid, b + hi, cmp); });
    }
    for (auto& x : th) x.join();
  }
}

// Elimination tree of the symmetric pattern in the new labels (Liu, path compression).
std::vector<int64_t> etree_sym(const Graph& g, const std::vector<int64_t>& q,
                               const std::vector<int64_t>& qinv) {
  int64_t n = g.n;
  std::vector<int64_t> parent(n, -1), anc(n, -1);
  for (int64_t j = 0; j < n; ++j) {
    int64_t u = q[j];
    for (int64_t e = g.ptr[u]; e < g.ptr[u + 1]; ++e) {
      int64_t i = qinv[g.adj[e]];
      if (i >= j) continue;
      // walk from i to the root of its current tree, compressing to j
      while (i != -1 && i < j) {
        int64_t nxt = anc[i];
        anc[i] = j;
        if (nxt == -1) { parent[i] = j; break; }
        i = nxt;
      }
    }
  }
  return parent;
}

std::vector<int64_t> postorder(const std::vector<int64_t>& parent) {
  int64_t n = (int64_t)parent.size();
  std::vector<int64_t> head(n, -1), next(n, -1), post;
  post.reserve(n);
  for (int64_t j = n - 1; j >= 0; --j) {
    if (parent[j] == -1) continue;
    next[j] = head[parent[j]];
    head[parent[j]] = j;
  }
  std::vector<int64_t> stack;
  for (int64_t r = 0; r < n; ++r) {
    if (parent[r] != -1) continue;
    stack.push_back(r);
    while (!stack.empty()) {
      int64_t p = stack.back();
      int64_t c = head[p];
      if (c == -1) {
        stack.pop_back();
        post.push_back(p);
      } else {
        head[p] = next[c];
        stack.push_back(c);
      }
    }
  }
  return post;
}

std::vector<int64_t> order_on_graph(int64_t n, const Graph& g, const PlanOptions& opt, std::string& err) {
  std::vector<int64_t> ord;
  if (opt.ordering == 1) {
    ord.resize(n);
    std::iota(ord.begin(), ord.end(), 0);
  } else if ((opt.ordering == 0 || opt.ordering == 2) && opt.grid[0] > 0 &&
             opt.grid[0] * std::max<int64_t>(opt.grid[1], 1) * std::max<int64_t>(opt.grid[2], 1) == n) {
    ord = order_geometric_nd(opt.grid[0], std::max<int64_t>(opt.grid[1], 1),
                             std::max<int64_t>(opt.grid[2], 1), opt.leaf_size);
  } else if (opt.ordering == 2) {
    err = "geometric ND needs grid[] with prod(grid) == n";
  } else if (opt.ordering == 5) {
    ord = order_amd(g);
  } else {
    ord = order_graph_nd(g, opt.leaf_size);
  }
  return ord;
}

}  // namespace

std::vector<int64_t> compute_order(int64_t n, const int64_t* colptr, const int32_t* rowval,
                                   const PlanOptions& opt, std::string& err) {
  Graph g = build_sym_graph(n, colptr, rowval);
  return order_on_graph(n, g, opt, err);
}

std::string Plan::build(int64_t n_, const int64_t* colptr, const int64_t* rowval, int base,
                        const PlanOptions& opt, const int64_t* pgiven, const int64_t* qgiven,
                        const int64_t* rowmatch) {
  auto t0 = std::chrono::steady_clock::now();
  auto tp = t0;
  auto phase = [&](int i) {
    const auto t = std::chrono::steady_clock::now();
    phase_ms[i] += std::chrono::duration<double, std::milli>(t - tp).count();
    tp = t;
  };
  n = n_;
  if (n <= 0) return "n must be positive";
  if (n >= (int64_t)INT32_MAX) return "n too large for int32 row indices";
  // ---- copy + validate input pattern ----
  Acolptr.assign(n + 1, 0);
  int64_t c0 = colptr[0] - base;
  if (c0 != 0) return "colptr[0] must equal index_base";
  for (int64_t j = 0; j <= n; ++j) Acolptr[j] = colptr[j] - base;
  nnzA = Acolptr[n];
  if (nnzA < 0) return "negative nnz";
  Arow.resize(nnzA);
  for (int64_t j = 0; j < n; ++j) {
    if (Acolptr[j + 1] < Acolptr[j]) return "colptr not monotone";
    int64_t prev = -1;
    for (int64_t e = Acolptr[j]; e < Acolptr[j + 1]; ++e) {
      int64_t r = rowval[e] - base;
      if (r < 0 || r >= n) return "row index out of range";
      if (r <= prev) return "row indices must be strictly increasing within a column";
      prev = r;
      Arow[e] = (int32_t)r;
    }
  }
  {   // is the pattern of A symmetric?  (the supernodal structure below is that of A+A')
    std::vector<int64_t> cnt(n + 1, 0);
    for (int64_t e = 0; e < nnzA; ++e) ++cnt[Arow[e] + 1];
    for (int64_t i = 0; i < n; ++i) cnt[i + 1] += cnt[i];
    sym_pattern = true;
    std::vector<int64_t> pos(cnt.begin(), cnt.end() - 1);
    std::vector<int32_t> tr(nnzA);
    for (int64_t j = 0; j < n; ++j)
      for (int64_t e = Acolptr[j]; e < Acolptr[j + 1]; ++e) tr[pos[Arow[e]]++] = (int32_t)j;
    for (int64_t j = 0; j <= n && sym_pattern; ++j) sym_pattern = cnt[j] == Acolptr[j];
    for (int64_t e = 0; e < nnzA && sym_pattern; ++e) sym_pattern = tr[e] == Arow[e];
  }
  phase(0);
  Graph g = build_sym_graph(n, Acolptr.data(), Arow.data());
  // Row pre-permutation from a transversal (match[c] = row of A placed at column c's
  // diagonal): the fronts are built on pattern(B + B') with B = A[match, :], labelled by columns.
  matched = rowmatch != nullptr && pgiven == nullptr;
  if (matched) {
    std::vector<int64_t> minv(n, -1);
    for (int64_t c = 0; c < n; ++c) {
      if (rowmatch[c] < 0 || rowmatch[c] >= n || minv[rowmatch[c]] >= 0) return "row match is not a permutation";
      minv[rowmatch[c]] = c;
    }
    std::vector<int64_t> bptr(n + 1, 0);
    std::vector<int32_t> brow(nnzA);
    for (int64_t c = 0; c < n; ++c) {
      for (int64_t e = Acolptr[c]; e < Acolptr[c + 1]; ++e) brow[e] = (int32_t)minv[Arow[e]];
      std::sort(brow.begin() + Acolptr[c], brow.begin() + Acolptr[c + 1]);
      bptr[c + 1] = Acolptr[c + 1];
    }
    g = build_sym_graph(n, bptr.data(), brow.data());
  }

  phase(1);
  // ---- ordering ----
  given_order = (pgiven != nullptr && qgiven != nullptr);
  std::vector<int64_t> ord;
  if (given_order) {
    ord.resize(n);
    for (int64_t k = 0; k < n; ++k) ord[k] = qgiven[k] - base;
  } else if (!opt.preorder.empty()) {
    ord = opt.preorder;
  } else {
    std::string err;
    ord = order_on_graph(n, g, opt, err);
    if (!err.empty()) return err;
  }
  if ((int64_t)ord.size() != n) return "ordering is not a permutation";
  {
    std::vector<char> seen(n, 0);
    for (auto v : ord) {
      if (v < 0 || v >= n || seen[v]) return "ordering is not a permutation";
      seen[v] = 1;
    }
  }
  // For a given (p, q), the symmetric pattern used is that of B + B' with B = A[p, q]:
  // build it in q-labels by mapping rows through p.
  if (given_order) {
    std::vector<int64_t> pv(n), pinv(n);
    for (int64_t k = 0; k < n; ++k) pv[k] = pgiven[k] - base;
    for (int64_t k = 0; k < n; ++k) {
      if (pv[k] < 0 || pv[k] >= n) return "p out of range";
      pinv[pv[k]] = k;
    }
    std::vector<int64_t> qinv_(n);
    for (int64_t k = 0; k < n; ++k) qinv_[ord[k]] = k;
    // B in new labels: entry (pinv[r], qinv[c]); relabel to "old" = ord[new] space so the
    // generic code below (which maps old->new via qinv) sees B's symmetric pattern.
    std::vector<int64_t> bptr(n + 1, 0);
    std::vector<int32_t> brow;
    std::vector<std::vector<int32_t>> cols(n);
    for (int64_t c = 0; c < n; ++c)
      for (int64_t e = Acolptr[c]; e < Acolptr[c + 1]; ++e)
        cols[c].push_back((int32_t)ord[pinv[Arow[e]]]);  // row mapped into q's label space
    for (int64_t c = 0; c < n; ++c) {
      std::sort(cols[c].begin(), cols[c].end());
      cols[c].erase(std::unique(cols[c].begin(), cols[c].end()), cols[c].end());
      bptr[c + 1] = bptr[c] + (int64_t)cols[c].size();
      brow.insert(brow.end(), cols[c].begin(), cols[c].end());
    }
    g = build_sym_graph(n, bptr.data(), brow.data());
    p0 = pv;
  }

  phase(2);
  q = ord;
  qinv.assign(n, 0);
  for (int64_t k = 0; k < n; ++k) qinv[q[k]] = k;

  // ---- elimination tree + postorder ----
  std::vector<int64_t> parent = etree_sym(g, q, qinv);
  if (!given_order) {
    // postorder: an equivalent order whose etree is the same tree relabelled (no second pass)
    std::vector<int64_t> post = postorder(parent);
    std::vector<int64_t> q2(n), pinv(n), parent2(n);
    for (int64_t k = 0; k < n; ++k) q2[k] = q[post[k]];
    for (int64_t k = 0; k < n; ++k) pinv[post[k]] = k;
    for (int64_t k = 0; k < n; ++k) parent2[k] = parent[post[k]] < 0 ? -1 : pinv[parent[post[k]]];
    q.swap(q2);
    parent.swap(parent2);
    for (int64_t k = 0; k < n; ++k) qinv[q[k]] = k;
  }
  if (!given_order) p0 = q;
  if (matched)
    for (int64_t k = 0; k < n; ++k) p0[k] = rowmatch[q[k]];
  p0inv.assign(n, 0);
  for (int64_t k = 0; k < n; ++k) p0inv[p0[k]] = k;

  phase(3);
  // ---- column counts (Gilbert-Ng-Peyton), labels are (post)ordered: parent > child ----
  std::vector<int64_t> cc(n, 0);
  {
    std::vector<int64_t> first(n), maxfirst(n, -1), prevleaf(n, -1), anc(n);
    std::vector<char> haschild(n, 0);
    for (int64_t j = 0; j < n; ++j) {
      first[j] = j;
      anc[j] = j;
    }
    for (int64_t j = 0; j < n; ++j)
      if (parent[j] != -1) {
        first[parent[j]] = std::min(first[parent[j]], first[j]);
        haschild[parent[j]] = 1;
      }
    // first[] must be the smallest label of the subtree; labels need not be a postorder for
    // given orders, so recompute by propagating in increasing label order (parent > child).
    for (int64_t j = 0; j < n; ++j) cc[j] = haschild[j] ? 0 : 1;
    // postorder <=> every subtree occupies the contiguous label range [first[j], j]
    bool is_post = true;
    {
      std::vector<int64_t> sz(n, 1);
      for (int64_t j = 0; j < n; ++j)
        if (parent[j] != -1) sz[parent[j]] += sz[j];
      for (int64_t j = 0; j < n && is_post; ++j)
        if (j - first[j] + 1 != sz[j]) is_post = false;
    }
    std::vector<int64_t> nbr;
    for (int64_t j = 0; j < n; ++j) {
      if (parent[j] != -1) cc[parent[j]]--;
      int64_t u = q[j];
      for (int64_t e = g.ptr[u]; e < g.ptr[u + 1]; ++e) {
        int64_t i = qinv[g.adj[e]];
        if (i <= j) continue;
        if (first[j] <= maxfirst[i]) continue;
        maxfirst[i] = first[j];
        int64_t jprev = prevleaf[i];
        prevleaf[i] = j;
        cc[j]++;
        if (jprev != -1) {
          int64_t qq = jprev;
          while (qq != anc[qq]) qq = anc[qq];
          for (int64_t s = jprev; s != qq;) {
            int64_t sp = anc[s];
            anc[s] = qq;
            s = sp;
          }
          cc[qq]--;
        }
      }
      if (parent[j] != -1) anc[j] = parent[j];
    }
    for (int64_t j = 0; j < n; ++j)
      if (parent[j] != -1) cc[parent[j]] += cc[j];
    if (!is_post) {
      // GNP needs a postorder; for given (non-postordered) orders fall back to the
      // row-structure computation below to obtain counts (cc recomputed there).
      std::fill(cc.begin(), cc.end(), -1);
    }
  }

  phase(4);
  // ---- exact supernodes: j, j+1 together iff parent[j]==j+1 && cc[j]==cc[j+1]+1 ----
  // For given non-postordered orders cc is unknown; compute exact structures column by
  // column with the symbolic "row structure" walk restricted to supernode detection.
  bool have_cc = cc[0] >= 0;
  t_first.clear();
  t_first.push_back(0);
  for (int64_t j = 0; j + 1 < n; ++j) {
    bool join = have_cc && parent[j] == j + 1 && cc[j] == cc[j + 1] + 1;
    if (!join) t_first.push_back(j + 1);
  }
  t_first.push_back(n);
  ntsup = (int64_t)t_first.size() - 1;
  col2t.assign(n, 0);
  for (int64_t t = 0; t < ntsup; ++t)
    for (int64_t j = t_first[t]; j < t_first[t + 1]; ++j) col2t[j] = (int32_t)t;
  // supernodal etree
  std::vector<int64_t> t_parent(ntsup, -1);
  for (int64_t t = 0; t < ntsup; ++t) {
    int64_t last = t_first[t + 1] - 1;
    if (parent[last] != -1) t_parent[t] = col2t[parent[last]];
  }
  // children lists of the supernodal tree
  std::vector<int64_t> tch_ptr(ntsup + 1, 0);
  std::vector<int32_t> tch;
  {
    std::vector<int64_t> cnt(ntsup, 0);
    for (int64_t t = 0; t < ntsup; ++t)
      if (t_parent[t] != -1) cnt[t_parent[t]]++;
    for (int64_t t = 0; t < ntsup; ++t) tch_ptr[t + 1] = tch_ptr[t] + cnt[t];
    tch.resize(tch_ptr[ntsup]);
    std::vector<int64_t> pos(tch_ptr.begin(), tch_ptr.end() - 1);
    for (int64_t t = 0; t < ntsup; ++t)
      if (t_parent[t] != -1) tch[pos[t_parent[t]]++] = (int32_t)t;
  }
  // row structures R_t = (union of A pattern of t's columns, rows > last) U (children R \ cols(t))
  if (have_cc) {
    // |R_t| = cc[last] - 1 is known: every t writes its own slice of t_rows, all t of one height
    // in the t-supernode tree at once (children are lower), thread-local marks
    t_rowptr.assign(ntsup + 1, 0);
    for (int64_t t = 0; t < ntsup; ++t) t_rowptr[t + 1] = t_rowptr[t] + (cc[t_first[t + 1] - 1] - 1);
    t_rows.assign(t_rowptr[ntsup], 0);
    std::vector<int32_t> height(ntsup, 0);
    int32_t hmax = 0;
    for (int64_t t = 0; t < ntsup; ++t) {
      for (int64_t k = tch_ptr[t]; k < tch_ptr[t + 1]; ++k) height[t] = std::max(height[t], height[tch[k]] + 1);
      hmax = std::max(hmax, height[t]);
    }
    std::vector<int64_t> hptr(hmax + 2, 0), hlist(ntsup);
    for (int64_t t = 0; t < ntsup; ++t) hptr[height[t] + 1]++;
    for (int32_t h2 = 0; h2 <= hmax; ++h2) hptr[h2 + 1] += hptr[h2];
    {
      std::vector<int64_t> pos(hptr.begin(), hptr.end() - 1);
      for (int64_t t = 0; t < ntsup; ++t) hlist[pos[height[t]]++] = t;
    }
    std::atomic<bool> bad{false};
    const int T = plan_threads();
    std::vector<std::vector<int32_t>> marks(T);
    std::atomic<int> slot{0};
    for (int32_t h2 = 0; h2 <= hmax; ++h2) {
      const int64_t lo0 = hptr[h2], cnt = hptr[h2 + 1] - hptr[h2];
      slot = 0;
      parallel_for(cnt, [&](int64_t lo, int64_t hi) {
        const int me = slot++;
        std::vector<int32_t>& mark = marks[me];
        if (mark.empty()) mark.assign(n, -1);
        std::vector<int32_t> buf;
        for (int64_t x = lo; x < hi; ++x) {
          const int64_t t = hlist[lo0 + x];
          const int64_t f = t_first[t], l = t_first[t + 1] - 1;
          buf.clear();
          for (int64_t j = f; j <= l; ++j) {
            int64_t u = q[j];
            for (int64_t e = g.ptr[u]; e < g.ptr[u + 1]; ++e) {
              int64_t i = qinv[g.adj[e]];
              if (i > l && mark[i] != (int32_t)t) { mark[i] = (int32_t)t; buf.push_back((int32_t)i); }
            }
          }
          for (int64_t k = tch_ptr[t]; k < tch_ptr[t + 1]; ++k) {
            int64_t c = tch[k];
            for (int64_t e = t_rowptr[c]; e < t_rowptr[c + 1]; ++e) {
              int64_t i = t_rows[e];
              if (i > l && mark[i] != (int32_t)t) { mark[i] = (int32_t)t; buf.push_back((int32_t)i); }
            }
          }
          if ((int64_t)buf.size() != t_rowptr[t + 1] - t_rowptr[t]) { bad = true; continue; }
          std::sort(buf.begin(), buf.end());
          std::copy(buf.begin(), buf.end(), t_rows.begin() + t_rowptr[t]);
        }
      }, 2048);
    }
    if (bad) return "internal: column count mismatch";
  } else {
    t_rowptr.assign(ntsup + 1, 0);
    t_rows.clear();
    std::vector<int64_t> mark(n, -1);
    std::vector<int32_t> buf;
    // supernodes in increasing label order: children (smaller labels) first
    for (int64_t t = 0; t < ntsup; ++t) {
      int64_t f = t_first[t], l = t_first[t + 1] - 1;
      buf.clear();
      for (int64_t j = f; j <= l; ++j) {
        int64_t u = q[j];
        for (int64_t e = g.ptr[u]; e < g.ptr[u + 1]; ++e) {
          int64_t i = qinv[g.adj[e]];
          if (i > l && mark[i] != t) { mark[i] = t; buf.push_back((int32_t)i); }
        }
      }
      for (int64_t k = tch_ptr[t]; k < tch_ptr[t + 1]; ++k) {
        int64_t c = tch[k];
        for (int64_t e = t_rowptr[c]; e < t_rowptr[c + 1]; ++e) {
          int64_t i = t_rows[e];
          if (i > l && mark[i] != t) { mark[i] = t; buf.push_back((int32_t)i); }
        }
      }
      std::sort(buf.begin(), buf.end());
      t_rows.insert(t_rows.end(), buf.begin(), buf.end());
      t_rowptr[t + 1] = (int64_t)t_rows.size();
      if (have_cc && (int64_t)buf.size() != cc[l] - 1) return "internal: column count mismatch";
    }
  }

  phase(5);
  // exact structural counts + update count
  nnzL = 0;
  upd = 0;
  for (int64_t t = 0; t < ntsup; ++t) {
    double ns_ = (double)(t_first[t + 1] - t_first[t]);
    double nu_ = (double)(t_rowptr[t + 1] - t_rowptr[t]);
    // column j (k-th of ns) has (ns - k) + nu entries incl. diagonal
    nnzL += ns_ * (ns_ + 1) / 2 + ns_ * nu_;
    for (int64_t k = 0; k < (int64_t)ns_; ++k) {
      double off = (ns_ - k - 1) + nu_;
      upd += off * off;
    }
  }
  nnzU = nnzL;  // symmetric structure; U's diagonal counted once here, L's unit diag too

  // ---- relaxed amalgamation (merge a supernode with the child that ends right before it) ----
  std::vector<int64_t> r_first, r_parent_t;   // relaxed supernodes built over t-supernodes
  std::vector<int64_t> t2r(ntsup);
  {
    // work arrays per current (merged) supernode keyed by its top t-supernode
    std::vector<int64_t> mfirst(ntsup), mns(ntsup), mzeros(ntsup, 0);
    std::vector<int64_t> top_of_t(ntsup);        // merged supernode containing t -> its top t
    for (int64_t t = 0; t < ntsup; ++t) {
      mfirst[t] = t_first[t];
      mns[t] = t_first[t + 1] - t_first[t];
      top_of_t[t] = t;
    }
    std::vector<char> absorbed(ntsup, 0);
    if (opt.relax) {
      for (int64_t t = 0; t < ntsup; ++t) {
        // candidate child: the supernode whose last column is first(t)-1
        if (t_first[t] == 0) continue;
        int64_t cprev = col2t[t_first[t] - 1];
        int64_t ctop = top_of_t[cprev];
        if (t_parent[cprev] != t) continue;  // must be a child
        // merged child covers [mfirst[ctop], t_first[t]) ; its rows structure R_cprev
        int64_t nsc = mns[ctop], nsp = mns[t];
        double nuc = (double)(t_rowptr[cprev + 1] - t_rowptr[cprev]);
        double nup = (double)(t_rowptr[t + 1] - t_rowptr[t]);
        double ntot = (double)(nsc + nsp);
        double merged = ntot * (ntot + 1) / 2 + ntot * nup;
        double orig = (double)nsc * (nsc + 1) / 2 + nsc * nuc + (double)nsp * (nsp + 1) / 2 + nsp * nup;
        double z = (double)mzeros[ctop] + (double)mzeros[t] + (merged - orig);
        double zf = z / merged;
        bool ok = (ntot <= 4) || (ntot <= 16 && zf < 0.8) || (ntot <= 48 && zf < 0.1) ||
                  (zf < 0.05);
        if (ntot > 4096) ok = false;
        if (!ok) continue;
        // merge ctop-chain into t
        mfirst[t] = mfirst[ctop];
        mns[t] = nsc + nsp;
        mzeros[t] = (int64_t)z;
        absorbed[ctop] = 1;
        // every t-supernode of the child chain now belongs to t
        for (int64_t j = mfirst[ctop]; j < t_first[t];) {
          int64_t tt = col2t[j];
          top_of_t[tt] = t;
          j = t_first[tt + 1];
        }
      }
    }
    for (int64_t t = 0; t < ntsup; ++t) {
      if (absorbed[t]) continue;
      // t is a top; check it is not absorbed later (top_of_t[t]==t means it is its own top)
      if (top_of_t[t] != t) continue;
      r_first.push_back(mfirst[t]);
      r_parent_t.push_back(t);
    }
    // sort relaxed supernodes by first column
    std::vector<int64_t> idx(r_first.size());
    std::iota(idx.begin(), idx.end(), 0);
    std::sort(idx.begin(), idx.end(), [&](int64_t a, int64_t b) { return r_first[a] < r_first[b]; });
    std::vector<int64_t> rf, rt;
    for (auto i : idx) { rf.push_back(r_first[i]); rt.push_back(r_parent_t[i]); }
    r_first.swap(rf);
    r_parent_t.swap(rt);   // top t-supernode of each relaxed supernode
  }
  phase(6);
  nsup = (int64_t)r_first.size();
  s_first.assign(nsup + 1, 0);
  for (int64_t s = 0; s < nsup; ++s) s_first[s] = r_first[s];
  s_first[nsup] = n;
  col2s.assign(n, 0);
  for (int64_t s = 0; s < nsup; ++s)
    for (int64_t j = s_first[s]; j < s_first[s + 1]; ++j) col2s[j] = (int32_t)s;
  for (int64_t s = 0; s < nsup; ++s)
    if (s_first[s + 1] - 1 != t_first[r_parent_t[s] + 1] - 1) return "internal: relaxed supernode boundary";
  // rows of relaxed supernode s = R of its top t-supernode
  s_rowptr.assign(nsup + 1, 0);
  s_rows.clear();
  s_parent.assign(nsup, -1);
  for (int64_t s = 0; s < nsup; ++s) {
    int64_t t = r_parent_t[s];
    s_rows.insert(s_rows.end(), t_rows.begin() + t_rowptr[t], t_rows.begin() + t_rowptr[t + 1]);
    s_rowptr[s + 1] = (int64_t)s_rows.size();
    int64_t last = s_first[s + 1] - 1;
    if (parent[last] != -1) s_parent[s] = col2s[parent[last]];
  }
  // sanity: update rows of s are inside parent's front
  for (int64_t s = 0; s < nsup; ++s) {
    int64_t pp = s_parent[s];
    for (int64_t e = s_rowptr[s]; e < s_rowptr[s + 1]; ++e) {
      if (pp < 0) return "internal: root with update rows";
      if (local_index(pp, s_rows[e]) < 0) return "internal: update row not in parent front";
    }
  }
  // children, ranks, levels
  ch_ptr.assign(nsup + 1, 0);
  {
    std::vector<int64_t> cnt(nsup, 0);
    for (int64_t s = 0; s < nsup; ++s)
      if (s_parent[s] >= 0) cnt[s_parent[s]]++;
    for (int64_t s = 0; s < nsup; ++s) ch_ptr[s + 1] = ch_ptr[s] + cnt[s];
    ch_list.assign(ch_ptr[nsup], 0);
    child_rank.assign(nsup, 0);
    std::vector<int64_t> pos(ch_ptr.begin(), ch_ptr.end() - 1);
    for (int64_t s = 0; s < nsup; ++s)
      if (s_parent[s] >= 0) {
        child_rank[s] = (int32_t)(pos[s_parent[s]] - ch_ptr[s_parent[s]]);
        ch_list[pos[s_parent[s]]++] = (int32_t)s;
      }
  }
  s_level.assign(nsup, 0);
  nlevels = 0;
  for (int64_t s = 0; s < nsup; ++s) {  // children have smaller indices than parents
    int lv = 0;
    for (int64_t k = ch_ptr[s]; k < ch_ptr[s + 1]; ++k) lv = std::max(lv, s_level[ch_list[k]] + 1);
    s_level[s] = lv;
    nlevels = std::max(nlevels, lv + 1);
  }
  for (int64_t s = 0; s < nsup; ++s)
    if (s_parent[s] >= 0 && s_parent[s] <= s) return "internal: parent index not after child";
  lev_ptr.assign(nlevels + 1, 0);
  for (int64_t s = 0; s < nsup; ++s) lev_ptr[s_level[s] + 1]++;
  for (int l = 0; l < nlevels; ++l) lev_ptr[l + 1] += lev_ptr[l];
  lev_sup.assign(nsup, 0);
  {
    std::vector<int64_t> pos(lev_ptr.begin(), lev_ptr.end() - 1);
    for (int64_t s = 0; s < nsup; ++s) lev_sup[pos[s_level[s]]++] = (int32_t)s;
  }
  // relmap (child update rows -> parent local indices; both sorted so a merge suffices)
  relmap.assign(s_rows.size(), 0);
  for (int64_t s = 0; s < nsup; ++s) {
    int64_t pp = s_parent[s];
    if (pp < 0) continue;
    int64_t pf = s_first[pp], pl = s_first[pp + 1], pns = pl - pf;
    int64_t k = s_rowptr[pp];
    for (int64_t e = s_rowptr[s]; e < s_rowptr[s + 1]; ++e) {
      int64_t gidx = s_rows[e];
      if (gidx < pl) { relmap[e] = (int32_t)(gidx - pf); continue; }
      while (k < s_rowptr[pp + 1] && s_rows[k] < gidx) ++k;
      if (k == s_rowptr[pp + 1] || s_rows[k] != gidx) return "internal: relmap";
      relmap[e] = (int32_t)(pns + (k - s_rowptr[pp]));
    }
  }

  phase(7);
  // ---- HBM layout ----
  auto align = [](int64_t x) { return (x + 15) & ~int64_t(15); };
  Loff.assign(nsup, 0);
  Uoff.assign(nsup, 0);
  lev_foff.assign(nlevels + 1, 0);
  front_flops.assign(nsup, 0.0);
  int64_t cur = 0;
  front_max = ns_max = nu_max = 0;
  stored = 0;
  flops = 0;
  for (int l = 0; l < nlevels; ++l) {
    lev_foff[l] = cur;
    for (int64_t k = lev_ptr[l]; k < lev_ptr[l + 1]; ++k) {
      int64_t s = lev_sup[k];
      int64_t a = ns(s), b = nu(s), m = a + b;
      Loff[s] = cur;
      cur = align(cur + m * a);
      Uoff[s] = cur;
      cur = align(cur + a * b);
      front_max = std::max(front_max, m);
      ns_max = std::max(ns_max, a);
      nu_max = std::max(nu_max, b);
      stored += (double)m * a + (double)a * b;
      // partial LU of an m x m front with a pivots: sum_k 2 (m-k-1)^2 + (m-k-1)
      double fa = (double)a, fm = (double)m;
      double sum_sq = 0;
      // closed form: sum_{k=0}^{a-1} (m-1-k)^2
      auto S2 = [](double x) { return x * (x + 1) * (2 * x + 1) / 6.0; };
      sum_sq = S2(fm - 1) - S2(fm - 1 - fa);
      double sum_l = fa * (fm - 1) - fa * (fa - 1) / 2;
      flops += 2 * sum_sq + sum_l;
      front_flops[s] = 2 * sum_sq + sum_l;
    }
  }
  lev_foff[nlevels] = cur;
  factor_size = cur;
  // scratch: one block per level; live from its level until its last consumer's level
  Foff.assign(nsup, -1);
  lev_soff.assign(nlevels, 0);
  lev_ssize.assign(nlevels, 0);
  {
    std::vector<int> lev_end(nlevels, -1);  // last level that reads this level's F22
    for (int l = 0; l < nlevels; ++l) {
      int64_t sz = 0;
      for (int64_t k = lev_ptr[l]; k < lev_ptr[l + 1]; ++k) {
        int64_t s = lev_sup[k];
        int64_t b = nu(s);
        if (b == 0) continue;
        Foff[s] = sz;
        sz = align(sz + b * b);
        lev_end[l] = std::max(lev_end[l], s_level[s_parent[s]]);
      }
      lev_ssize[l] = sz;
    }
    // first-fit over [offset, size) intervals alive at the same time
    struct Blk { int64_t off, size; int end; };
    std::vector<Blk> live;
    int64_t peak = 0;
    for (int l = 0; l < nlevels; ++l) {
      // free blocks whose last consumer level < l
      live.erase(std::remove_if(live.begin(), live.end(), [&](const Blk& b) { return b.end < l; }),
                 live.end());
      if (lev_ssize[l] == 0) continue;
      std::sort(live.begin(), live.end(), [](const Blk& a, const Blk& b) { return a.off < b.off; });
      int64_t pos = 0;
      for (auto& b : live) {
        if (b.off - pos >= lev_ssize[l]) break;
        pos = std::max(pos, b.off + b.size);
      }
      lev_soff[l] = pos;
      live.push_back({pos, lev_ssize[l], lev_end[l]});
      peak = std::max(peak, pos + lev_ssize[l]);
    }
    scratch_size = peak;
    for (int64_t s = 0; s < nsup; ++s)
      if (Foff[s] >= 0) Foff[s] += lev_soff[s_level[s]];
  }

  phase(8);
  // ---- A map ----
  Adest.assign(nnzA, 0);
  A_s.assign(nnzA, 0);
  A_li.assign(nnzA, 0);
  A_lj.assign(nnzA, 0);
  std::vector<int> ent_level(nnzA, 0);
  {
    std::atomic<bool> outside{false};
    parallel_for(n, [&](int64_t c0, int64_t c1) {
      for (int64_t c = c0; c < c1; ++c) {
        int64_t pc = qinv[c];
        for (int64_t e = Acolptr[c]; e < Acolptr[c + 1]; ++e) {
          int64_t pr = p0inv[Arow[e]];
          int64_t k = std::min(pr, pc);
          int64_t s = col2s[k];
          int64_t li = local_index(s, pr), lj = local_index(s, pc);
          if (li < 0 || lj < 0) { outside = true; continue; }
          int64_t a = ns(s), m = M(s);
          int64_t dest;
          if (lj < a) dest = Loff[s] + lj * m + li;
          else if (li < a) dest = Uoff[s] + (lj - a) * a + li;
          else dest = -1 - (Foff[s] + (lj - a) * (m - a) + (li - a));
          Adest[e] = dest;
          A_s[e] = (int32_t)s;
          A_li[e] = (int32_t)li;
          A_lj[e] = (int32_t)lj;
          ent_level[e] = s_level[s];
        }
      }
    }, 4096);
    if (outside) return "internal: A entry outside its front";
  }
  {
    const auto t = std::chrono::steady_clock::now();
    phase_ms[10] += std::chrono::duration<double, std::milli>(t - tp).count();
  }
  Alev_ptr.assign(nlevels + 1, 0);
  for (int64_t e = 0; e < nnzA; ++e) Alev_ptr[ent_level[e] + 1]++;
  for (int l = 0; l < nlevels; ++l) Alev_ptr[l + 1] += Alev_ptr[l];
  Alev_ent.assign(nnzA, 0);
  {
    std::vector<int64_t> pos(Alev_ptr.begin(), Alev_ptr.end() - 1);
    for (int64_t e = 0; e < nnzA; ++e) Alev_ent[pos[ent_level[e]]++] = (int32_t)e;
    // front slots are distinct: a strict order, so the parallel sort equals std::sort
    const auto ts = std::chrono::steady_clock::now();
    // sorted as (key, entry) records: the comparator touches contiguous memory only
    std::vector<std::pair<int64_t, int32_t>> kv;
    for (int l = 0; l < nlevels; ++l) {
      const int64_t lo = Alev_ptr[l], cnt = Alev_ptr[l + 1] - lo;
      kv.resize((size_t)cnt);
      parallel_for(cnt, [&](int64_t a, int64_t b) {
        for (int64_t i = a; i < b; ++i) kv[i] = {Adest[Alev_ent[lo + i]], Alev_ent[lo + i]};
      });
      parallel_sort(kv.begin(), kv.end(), [](const std::pair<int64_t, int32_t>& a, const std::pair<int64_t, int32_t>& b) {
        return a.first < b.first;
      });
      parallel_for(cnt, [&](int64_t a, int64_t b) {
        for (int64_t i = a; i < b; ++i) Alev_ent[lo + i] = kv[i].second;
      });
    }
    phase_ms[11] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - ts).count();
  }
  // rows of A (for the row scaling kernel)
  Arowptr.assign(n + 1, 0);
  for (int64_t e = 0; e < nnzA; ++e) Arowptr[Arow[e] + 1]++;
  for (int64_t i = 0; i < n; ++i) Arowptr[i + 1] += Arowptr[i];
  Arow_ent.assign(nnzA, 0);
  {
    std::vector<int64_t> pos(Arowptr.begin(), Arowptr.end() - 1);
    for (int64_t c = 0; c < n; ++c)
      for (int64_t e = Acolptr[c]; e < Acolptr[c + 1]; ++e) Arow_ent[pos[Arow[e]]++] = (int32_t)e;
  }
  phase(9);
  analysis_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return "";
}

// ---------------------------------------------------------------------------------------
// Multi-GPU partition of the assembly tree: proportional mapping.  A set of subtrees is mapped onto
// a contiguous rank range [r0, r1): one rank takes them all; a single subtree on several ranks
// makes its root a shared ("top") front of the whole range and maps its children onto the same
// range; several subtrees are packed into bins whose rank counts follow their work (below).  Sibling
// shared fronts therefore have DISJOINT rank groups and run concurrently, and every group is a
// contiguous range (nested or disjoint: a rank belongs to at most one shared front per tree level).
// (Rounds 1-3 bin-packed the subtrees onto ranks, which put one rank under several siblings and
// serialised their shared fronts: 2.70x projected at 128^3 on 8 ranks, SMLU_PARTITION=binpack.)
// ---------------------------------------------------------------------------------------
void Plan::compute_owners(int np, int64_t block) {
  nparts = std::max(1, np);
  dob = std::max<int64_t>(64, (block / 64) * 64);
  owner.assign(nsup, 0);
  group.assign(nsup, std::vector<int32_t>{0});
  if (nparts == 1 || nsup == 0) return;
  std::vector<double> W(front_flops.begin(), front_flops.end());   // subtree work
  for (int64_t s = 0; s < nsup; ++s)
    if (s_parent[s] >= 0) W[s_parent[s]] += W[s];
  std::vector<char> top(nsup, 0);
  std::vector<int32_t> sub_owner(nsup, -1);
  constexpr bool binpack = false;   // rounds 1-3's bin-packing, kept for the record
  if (!binpack) {
    std::vector<int32_t> lo(nsup, -1), hi(nsup, -1);   // rank range of each top front
    // Cost model of a subtree set on k ranks (flop units): one rank does all of it; a single
    // subtree shares its root front over the k ranks (front flops / k) and maps its children on
    // the same k ranks; several subtrees take the best bin split.  A split deals the ranks one at
    // a time to the bin of largest cost at its current count (a bin whose subtrees cannot use
    // more ranks -- one leaf -- stops gaining), so it sees that a heavy subtree left on one rank
    // bounds the makespan, which plain work-proportional shares do not.
    std::map<std::pair<int64_t, int>, double> memo;
    std::function<double(const std::vector<int64_t>&, int)> cost;
    std::function<double(const std::vector<int64_t>&, int, std::vector<int>*, std::vector<int>*)> split;
    cost = [&](const std::vector<int64_t>& S, int k) -> double {
      double w = 0;
      for (auto v : S) w += W[v];
      if (k <= 1 || S.empty()) return w;
      if (S.size() == 1) {
        const int64_t v = S[0];
        if (ch_ptr[v] == ch_ptr[v + 1]) return w;
        auto key = std::make_pair(v, k);
        auto it = memo.find(key);
        if (it != memo.end()) return it->second;
        std::vector<int64_t> ch(ch_list.begin() + ch_ptr[v], ch_list.begin() + ch_ptr[v + 1]);
        std::sort(ch.begin(), ch.end(), [&](int64_t a, int64_t b) { return W[a] != W[b] ? W[a] > W[b] : a < b; });
        const double c = front_flops[v] / k + cost(ch, k);
        memo[key] = c;
        return c;
      }
      return split(S, k, nullptr, nullptr);
    };
    split = [&](const std::vector<int64_t>& S, int k, std::vector<int>* obin, std::vector<int>* orank) -> double {
      const int mmax = (int)std::min<size_t>(S.size(), (size_t)k);
      // m = 1: the heaviest subtree (S is sorted) on all k ranks, the light rest packed whole onto the
      // range's first rank (bin -1), which also works on the heavy one: no rank is taken from it
      double best;
      {
        double rest = 0;
        for (size_t i = 1; i < S.size(); ++i) rest += W[S[i]];
        best = cost(std::vector<int64_t>{S[0]}, k) + rest;
        if (obin) {
          obin->assign(S.size(), -1);
          (*obin)[0] = 0;
        }
        if (orank) orank->assign(1, k);
      }
      for (int m = 2; m <= mmax; ++m) {
        std::vector<double> bw(m, 0.0);
        std::vector<int> bin(S.size());
        std::vector<std::vector<int64_t>> sets(m);
        for (size_t i = 0; i < S.size(); ++i) {
          const int b = (int)(std::min_element(bw.begin(), bw.end()) - bw.begin());
          bin[i] = b;
          bw[b] += W[S[i]];
          sets[b].push_back(S[i]);
        }
        std::vector<int> r(m, 1);
        std::vector<double> c(m);
        for (int b = 0; b < m; ++b) c[b] = cost(sets[b], 1);
        for (int extra = k - m; extra > 0; --extra) {
          // the most expensive bin that still gains from one more rank (a single leaf does not)
          std::vector<int> ord(m);
          std::iota(ord.begin(), ord.end(), 0);
          std::sort(ord.begin(), ord.end(), [&](int a, int b) { return c[a] != c[b] ? c[a] > c[b] : a < b; });
          int bi = ord[0];
          double cb = cost(sets[bi], r[bi] + 1);
          for (int o : ord) {
            const double cn = cost(sets[o], r[o] + 1);
            if (cn < c[o] * (1 - 1e-12)) { bi = o; cb = cn; break; }
          }
          ++r[bi];
          c[bi] = cb;
        }
        const double mk = *std::max_element(c.begin(), c.end());
        if (best < 0 || mk < best * (1 - 1e-12)) {
          best = mk;
          if (obin) *obin = bin;
          if (orank) *orank = r;
        }
      }
      return best;
    };
    struct Job { std::vector<int64_t> sub; int r0, r1; };
    std::vector<Job> stack;
    {
      Job j{{}, 0, nparts};
      for (int64_t s = 0; s < nsup; ++s)
        if (s_parent[s] < 0) j.sub.push_back(s);
      stack.push_back(std::move(j));
    }
    while (!stack.empty()) {
      Job j = std::move(stack.back());
      stack.pop_back();
      if (j.sub.empty()) continue;
      if (j.r1 - j.r0 == 1) {
        for (auto v : j.sub) sub_owner[v] = j.r0;
        continue;
      }
      constexpr bool dbg = false;
      if (dbg && j.r1 - j.r0 >= 2) {
        std::fprintf(stderr, "map ranks [%d,%d):", j.r0, j.r1);
        for (auto v : j.sub) std::fprintf(stderr, " %lld(W %.3e ns %lld)", (long long)v, W[v], (long long)ns(v));
        std::fprintf(stderr, "\n");
      }
      if (j.sub.size() == 1) {
        const int64_t v = j.sub[0];
        if (ch_ptr[v] == ch_ptr[v + 1]) {   // a leaf front cannot be split further
          sub_owner[v] = j.r0;
          continue;
        }
        top[v] = 1;
        lo[v] = j.r0;
        hi[v] = j.r1;
        Job c{{}, j.r0, j.r1};
        for (int64_t e = ch_ptr[v]; e < ch_ptr[v + 1]; ++e) c.sub.push_back(ch_list[e]);
        stack.push_back(std::move(c));
        continue;
      }
      // several subtrees on k ranks: pack them into m bins (largest first onto the lightest bin) and
      // deal the ranks to the bins by the cost model below; keep the m (2 <= m <= k) of smallest
      // makespan.  Every bin becomes a job on its own contiguous rank range.
      std::sort(j.sub.begin(), j.sub.end(), [&](int64_t a, int64_t b) { return W[a] != W[b] ? W[a] > W[b] : a < b; });
      std::vector<int> bin, r;
      split(j.sub, j.r1 - j.r0, &bin, &r);
      for (size_t i = 0; i < j.sub.size(); ++i)
        if (bin[i] < 0) sub_owner[j.sub[i]] = j.r0;   // light subtrees packed onto the first rank
      int r0 = j.r0;
      for (size_t b = 0; b < r.size(); ++b) {
        Job c{{}, r0, r0 + r[b]};
        for (size_t i = 0; i < j.sub.size(); ++i)
          if (bin[i] == (int)b) c.sub.push_back(j.sub[i]);
        r0 += r[b];
        stack.push_back(std::move(c));
      }
    }
    for (int64_t s = nsup - 1; s >= 0; --s) {   // parents before children
      if (top[s]) continue;
      if (sub_owner[s] >= 0) owner[s] = sub_owner[s];
      else if (s_parent[s] >= 0) owner[s] = owner[s_parent[s]];
    }
    for (int64_t s = 0; s < nsup; ++s) {
      if (!top[s]) {
        group[s].assign(1, owner[s]);
        continue;
      }
      group[s].clear();
      for (int r = lo[s]; r < hi[s]; ++r) group[s].push_back(r);
      owner[s] = -1;
    }
    return;
  }
  // bin-packing (rounds 1-3, kept for comparison): split the heaviest subtree into its children
  // until every subtree fits the per-rank share, bin-pack the subtrees (largest first, least-loaded
  // rank); a top front's group is the union of its children's groups
  std::vector<int64_t> S;
  for (int64_t s = 0; s < nsup; ++s)
    if (s_parent[s] < 0) S.push_back(s);
  auto heaviest = [&]() {
    size_t bi = 0;
    for (size_t i = 1; i < S.size(); ++i)
      if (W[S[i]] > W[S[bi]]) bi = i;
    return bi;
  };
  for (int it = 0; it < 64 * nparts && !S.empty(); ++it) {
    double sub = 0;
    for (auto v : S) sub += W[v];
    const size_t bi = heaviest();
    const int64_t v = S[bi];
    if ((int)S.size() >= nparts && W[v] <= 1.05 * sub / nparts) break;
    if (ch_ptr[v] == ch_ptr[v + 1]) break;
    top[v] = 1;
    S.erase(S.begin() + (long)bi);
    for (int64_t e = ch_ptr[v]; e < ch_ptr[v + 1]; ++e) S.push_back(ch_list[e]);
  }
  std::sort(S.begin(), S.end(), [&](int64_t a, int64_t b) { return W[a] != W[b] ? W[a] > W[b] : a < b; });
  std::vector<double> load(nparts, 0.0);
  for (auto v : S) {
    const int r = (int)(std::min_element(load.begin(), load.end()) - load.begin());
    load[r] += W[v];
    sub_owner[v] = r;
  }
  for (int64_t s = nsup - 1; s >= 0; --s) {
    if (sub_owner[s] >= 0) owner[s] = sub_owner[s];
    else if (!top[s] && s_parent[s] >= 0) owner[s] = owner[s_parent[s]];
  }
  for (int64_t s = 0; s < nsup; ++s) {
    if (!top[s]) {
      group[s].assign(1, owner[s]);
      continue;
    }
    std::vector<int32_t> g;
    for (int64_t e = ch_ptr[s]; e < ch_ptr[s + 1]; ++e)
      g.insert(g.end(), group[ch_list[e]].begin(), group[ch_list[e]].end());
    std::sort(g.begin(), g.end());
    g.erase(std::unique(g.begin(), g.end()), g.end());
    group[s] = g;
    owner[s] = g.size() == 1 ? g[0] : -1;
  }
}

namespace {
// first-fit allocation of blocks live over level intervals [lo, hi]
struct LiveAlloc {
  struct Blk { int64_t off, size; int hi; };
  std::vector<Blk> live;
  int64_t peak = 0;
  void release_before(int l) {
    live.erase(std::remove_if(live.begin(), live.end(), [&](const Blk& b) { return b.hi < l; }), live.end());
  }
  int64_t take(int64_t size, int hi) {
    if (size <= 0) return -1;
    std::sort(live.begin(), live.end(), [](const Blk& a, const Blk& b) { return a.off < b.off; });
    int64_t pos = 0;
    for (auto& b : live) {
      if (b.off - pos >= size) break;
      pos = std::max(pos, b.off + b.size);
    }
    live.push_back({pos, size, hi});
    peak = std::max(peak, pos + size);
    return pos;
  }
};
int64_t al16(int64_t x) { return (x + 15) & ~int64_t(15); }
}  // namespace

void rank_layout(const Plan& P, int r, RankLayout& L) {
  L = RankLayout();
  L.rank = r;
  const int64_t nsup = P.nsup;
  L.Loff.assign(nsup, -1);
  L.Uoff.assign(nsup, -1);
  L.Foff.assign(nsup, -1);
  L.recv_off.assign(nsup, -1);
  L.recv_size.assign(nsup, 0);
  auto member = [&](int64_t s) {
    return std::binary_search(P.group[s].begin(), P.group[s].end(), (int32_t)r);
  };
  // factor store
  int64_t cur = 0;
  for (int l = 0; l < P.nlevels; ++l)
    for (int64_t k = P.lev_ptr[l]; k < P.lev_ptr[l + 1]; ++k) {
      const int64_t s = P.lev_sup[k];
      const int64_t a = P.ns(s), m = P.M(s);
      if (!P.dist(s)) {
        if (P.owner[s] != r) continue;
        L.Loff[s] = cur;
        cur = al16(cur + m * a);
        L.Uoff[s] = cur;
        cur = al16(cur + a * P.nu(s));
        continue;
      }
      if (!member(s)) continue;
      const int64_t nb = P.npblk(s) + P.nublk(s);
      for (int64_t b = 0; b < nb; ++b) {
        if (P.blk_owner(s, b) != r) continue;
        RankLayout::Blk B{(int32_t)s, (int32_t)b, P.blk_c0(s, b), P.blk_c1(s, b), cur, -1};
        const int64_t w = B.c1 - B.c0;
        cur = al16(cur + (b < P.npblk(s) ? m : a) * w);
        L.blocks.push_back(B);
      }
      L.stage_size = std::max(L.stage_size, m * P.dob);
    }
  L.store_size = cur;
  // scratch: per level, the F22 rows of this rank's fronts (live until the parents' level) and
  // the receive areas of its distributed fronts (live at their level)
  LiveAlloc A;
  for (int l = 0; l < P.nlevels; ++l) {
    A.release_before(l);
    int64_t sz = 0;
    int hi = -1;
    std::vector<std::pair<int64_t*, int64_t>> place;   // (slot, offset within the level block)
    for (int64_t k = P.lev_ptr[l]; k < P.lev_ptr[l + 1]; ++k) {
      const int64_t s = P.lev_sup[k];
      const int64_t b = P.nu(s);
      if (b == 0 || P.s_parent[s] < 0) continue;
      if (!P.dist(s)) {
        if (P.owner[s] != r) continue;
        place.push_back({&L.Foff[s], sz});
        sz = al16(sz + b * b);
      } else {
        if (!member(s)) continue;
        for (auto& B : L.blocks)
          if (B.s == s && B.c0 >= P.ns(s)) {
            place.push_back({&B.foff, sz});
            sz = al16(sz + b * (B.c1 - B.c0));
          }
      }
      hi = std::max(hi, (int)P.s_level[P.s_parent[s]]);
    }
    if (sz > 0) {
      const int64_t base = A.take(sz, hi);
      for (auto& pl : place) *pl.first = base + pl.second;
    }
    // receive areas of the distributed fronts at this level
    for (int64_t k = P.lev_ptr[l]; k < P.lev_ptr[l + 1]; ++k) {
      const int64_t t = P.lev_sup[k];
      if (!P.dist(t) || !member(t)) continue;
      int64_t need = 0;
      for (int64_t e = P.ch_ptr[t]; e < P.ch_ptr[t + 1]; ++e) {
        const int64_t c = P.ch_list[e];
        const int64_t nuc = P.nu(c);
        const int32_t* rm = P.relmap.data() + P.s_rowptr[c];
        for (int64_t jc = 0; jc < nuc; ++jc)
          if (P.col_owner(t, rm[jc]) == r && P.col_owner(c, P.ns(c) + jc) != r) need += nuc;
      }
      L.recv_size[t] = need;
      if (need > 0) L.recv_off[t] = A.take(al16(need), l);
    }
  }
  L.scratch_size = A.peak;
}

double project_partition(const Plan& P, double tflops, double gbs, double lat_us, double* t1_out) {
  const double rate = tflops * 1e12, bw = gbs * 1e9, lat = lat_us * 1e-6;
  // calibrated on one MI355X (round 5): 80 us per 64-column panel step (panel, inverses, TRSM,
  // in-block update: 695 steps ~ 56 ms at 128^3), 0.32 ms per level (launch latencies, the small
  // fronts' kernels and the per-refactor dominance check: C2 7.9 ms over 18 levels), and the
  // caller's rate for the dense front work (52 TFLOP/s reproduces 0.49 s at 128^3 with both)
  const double step_lat = 80e-6;
  const double level_lat = 0.32e-3;
  auto panel_chain = [&](int64_t s) { return P.ns(s) > 128 ? step_lat * (double)((P.ns(s) + 63) / 64) : 0.0; };
  // The fronts of one level that one GPU owns run batched (every launch of the level covers all of
  // them, in lockstep): their dense work adds up, their panel chains overlap, so a level costs
  // sum(flops) / rate + max(chain) on that GPU (round 4 summed the chains: 0.80 s projected at
  // 128^3 against 0.49-0.50 s measured).
  double t1 = 0;
  for (int l = 0; l < P.nlevels; ++l) {
    double fl = 0, ch = 0;
    for (int64_t k = P.lev_ptr[l]; k < P.lev_ptr[l + 1]; ++k) {
      fl += P.front_flops[P.lev_sup[k]];
      ch = std::max(ch, panel_chain(P.lev_sup[k]));
    }
    t1 += fl / rate + ch + level_lat;
  }
  if (t1_out) *t1_out = t1;
  std::vector<double> clk(P.nparts, 0.0);
  std::vector<double> lev_fl(P.nparts), lev_ch(P.nparts);
  for (int l = 0; l < P.nlevels; ++l) {
    std::fill(lev_fl.begin(), lev_fl.end(), 0.0);
    std::fill(lev_ch.begin(), lev_ch.end(), 0.0);
    for (int64_t k = P.lev_ptr[l]; k < P.lev_ptr[l + 1]; ++k) {
      const int64_t s = P.lev_sup[k];
      if (P.dist(s)) continue;
      lev_fl[P.owner[s]] += P.front_flops[s];
      lev_ch[P.owner[s]] = std::max(lev_ch[P.owner[s]], panel_chain(s));
    }
    for (int r = 0; r < P.nparts; ++r) clk[r] += lev_fl[r] / rate + lev_ch[r] + level_lat;
    for (int64_t k = P.lev_ptr[l]; k < P.lev_ptr[l + 1]; ++k) {
      const int64_t s = P.lev_sup[k];
      if (!P.dist(s)) continue;
      const auto& G = P.group[s];
      double t = 0;
      for (int r : G) t = std::max(t, clk[r]);
      // children's F22 columns: each column to its owner (about all of them cross ranks)
      double xbytes = 0;
      for (int64_t e = P.ch_ptr[s]; e < P.ch_ptr[s + 1]; ++e)
        xbytes += 8.0 * (double)P.nu(P.ch_list[e]) * (double)P.nu(P.ch_list[e]);
      t += lat + xbytes / G.size() / bw;
      const double M = (double)P.M(s);
      const int64_t np = P.npblk(s), nb = np + P.nublk(s);
      // per-member clocks through the block-cyclic factorization with depth-1 look-ahead (the
      // schedule of build_schedule): the owner of pivot block b+1 applies b to block b+1 only,
      // factors b+1 and broadcasts it; it applies b to its other blocks after that broadcast
      std::map<int, double> c, pend;
      for (int r : G) { c[r] = t; pend[r] = 0.0; }
      constexpr bool la = false;   // the schedule's depth-1 look-ahead is off
      for (int64_t b = 0; b < np; ++b) {
        const double c0 = (double)P.blk_c0(s, b), c1 = (double)P.blk_c1(s, b), w = c1 - c0;
        const int o = P.blk_owner(s, b);
        const double inner = 2.0 * (M - c0) * w * w / rate + step_lat * std::ceil(w / 64.0);
        const double bcast = lat + 8.0 * (M - c0) * w / bw;
        double ready = c[o] + inner;
        for (int r : G)
          if (r != o) ready = std::max(ready, c[r]);
        const double tb = ready + bcast;
        const int nxt = (la && b + 1 < np) ? P.blk_owner(s, b + 1) : -1;
        for (int r : G) {   // trailing update of r's blocks right of this one
          double cols = 0, first = 0;
          for (int64_t bb = b + 1; bb < nb; ++bb)
            if (P.blk_owner(s, bb) == r) {
              const double wc = (double)(P.blk_c1(s, bb) - P.blk_c0(s, bb));
              cols += wc;
              if (bb == b + 1) first = wc;
            }
          const double upd = 2.0 * (M - c0) * w * cols / rate, upd1 = 2.0 * (M - c0) * w * first / rate;
          double cr = tb + pend[r];
          pend[r] = 0.0;
          if (r == nxt) {
            cr += upd1;
            pend[r] = upd - upd1;
          } else {
            cr += upd;
          }
          c[r] = cr;
        }
      }
      double tend = 0;
      for (int r : G) tend = std::max(tend, c[r] + pend[r]);
      constexpr bool dbg = false;
      if (dbg)
        std::fprintf(stderr, "shared front %lld level %d ns %lld M %lld group %zu: start %.4f end %.4f (flops %.3e)\n",
                     (long long)s, l, (long long)P.ns(s), (long long)P.M(s), G.size(), t, tend, P.front_flops[s]);
      for (int r : G) clk[r] = tend;
    }
  }
  return *std::max_element(clk.begin(), clk.end());
}

}  // namespace smlu
