// amd.cpp — approximate minimum degree ordering of the pattern of A+A' (SMLU_ORDER_AMD).
//
// The reference's column order comes from UMFPACK, whose symmetric strategy orders A+A' with AMD
// (reached through lu(A) at src/SharedMemSparseLU.jl:74).  This is a from-scratch restatement of
// the published algorithm (Amestoy, Davis & Duff, "An approximate minimum degree ordering
// algorithm", SIAM J. Matrix Anal. Appl. 17(4), 1996), not a port of any implementation:
//   * quotient graph: every uneliminated variable i keeps its adjacent elements E_i and its
//     adjacent variables A_i; every element e keeps its variable list L_e;
//   * the pivot p of minimum approximate external degree becomes an element with
//     L_p = (A_p u U_{e in E_p} L_e) \ {p}; the elements in E_p are absorbed into p;
//   * approximate external degree of i in L_p (weighted by supervariable sizes):
//       d_i = min(n - k - |i|, d_i_old + |L_p \ i|, |A_i \ L_p| + |L_p \ i| + sum_{e in E_i, e != p} |L_e \ L_p|),
//     with |L_e \ L_p| from one pass over L_p ("w(e)"); an element with |L_e \ L_p| = 0 is
//     absorbed into p (aggressive absorption);
//   * variables whose only neighbour is element p are eliminated with p (mass elimination);
//     variables of L_p with identical (E_i, A_i) merge into one supervariable (hash + compare).
// Not included: the dense-row pre-pass and AMD's exact tie-breaking, so the permutation is an
// AMD ordering but not UMFPACK's bit-for-bit (parity for the pivot order itself stays with the
// given-(p, q) hand-over, SMLU_ORDER_GIVEN).  Output: perm (new -> old), principal variables in
// elimination order, each followed by the variables merged into or mass-eliminated with it; the
// plan postorders the resulting elimination tree.
#include <algorithm>
#include <cstdint>
#include <vector>

#include "plan.hpp"

namespace smlu {

std::vector<int64_t> order_amd(const Graph& g) {
  const int64_t n = g.n;
  std::vector<int64_t> perm;
  perm.reserve(n);
  if (n == 0) return perm;
  enum : uint8_t { VAR = 0, ELEM = 1, DEAD = 2 };
  std::vector<uint8_t> st(n, VAR);
  std::vector<int64_t> nv(n, 1);                    // supervariable weight (0: not principal)
  std::vector<std::vector<int32_t>> E(n), A(n), L(n);
  std::vector<int64_t> deg(n), ew(n, 0);            // approximate external degree, |L_e| weighted
  for (int64_t i = 0; i < n; ++i) {
    A[i].assign(g.adj.begin() + g.ptr[i], g.adj.begin() + g.ptr[i + 1]);
    deg[i] = (int64_t)A[i].size();
  }
  // degree buckets (doubly linked lists)
  std::vector<int64_t> head(n + 1, -1), nxt(n, -1), prv(n, -1);
  auto ins = [&](int64_t i) {
    const int64_t d = deg[i];
    nxt[i] = head[d];
    prv[i] = -1;
    if (head[d] >= 0) prv[head[d]] = i;
    head[d] = i;
  };
  auto rem = [&](int64_t i) {
    if (prv[i] >= 0) nxt[prv[i]] = nxt[i];
    else head[deg[i]] = nxt[i];
    if (nxt[i] >= 0) prv[nxt[i]] = prv[i];
  };
  for (int64_t i = 0; i < n; ++i) ins(i);
  // output groups: principal -> linked list of the variables eliminated with it
  std::vector<int64_t> gnext(n, -1), gtail(n);
  for (int64_t i = 0; i < n; ++i) gtail[i] = i;
  auto join = [&](int64_t i, int64_t j) {   // append j's group to i's
    gnext[gtail[i]] = j;
    gtail[i] = gtail[j];
  };
  std::vector<int64_t> mark(n, 0), mark2(n, 0), w(n, 0);
  int64_t stamp = 0, stamp2 = 0, wflg = 1;
  std::vector<int32_t> Lp, keep;
  std::vector<std::pair<uint64_t, int32_t>> hv;
  int64_t nel = 0, mindeg = 0;
  while (nel < n) {
    while (mindeg <= n && head[mindeg] < 0) ++mindeg;
    const int64_t p = head[mindeg];
    rem(p);
    nel += nv[p];
    // ---- new element L_p ----
    mark[p] = ++stamp;
    Lp.clear();
    for (int32_t e : E[p]) {
      if (st[e] != ELEM) continue;
      for (int32_t i : L[e])
        if (nv[i] > 0 && st[i] == VAR && mark[i] != stamp) {
          mark[i] = stamp;
          Lp.push_back(i);
        }
      st[e] = DEAD;   // absorbed into p
      std::vector<int32_t>().swap(L[e]);
    }
    for (int32_t i : A[p])
      if (nv[i] > 0 && st[i] == VAR && mark[i] != stamp) {
        mark[i] = stamp;
        Lp.push_back(i);
      }
    std::vector<int32_t>().swap(E[p]);
    std::vector<int32_t>().swap(A[p]);
    st[p] = ELEM;
    int64_t degme = 0;
    for (int32_t i : Lp) {
      degme += nv[i];
      rem(i);
    }
    // ---- |L_e \ L_p| for the elements adjacent to L_p ----
    for (int32_t i : Lp)
      for (int32_t e : E[i]) {
        if (st[e] != ELEM) continue;
        if (w[e] < wflg) w[e] = ew[e] + wflg;
        w[e] -= nv[i];
      }
    // ---- prune lists, approximate degrees, mass elimination ----
    hv.clear();
    for (int32_t i : Lp) {
      int64_t d = 0;
      uint64_t h = 0;
      keep.clear();
      for (int32_t e : E[i]) {
        if (st[e] != ELEM) continue;
        const int64_t ext = w[e] - wflg;
        if (ext == 0) {               // L_e within L_p: aggressive absorption into p
          st[e] = DEAD;
          std::vector<int32_t>().swap(L[e]);
          continue;
        }
        d += ext;
        h += (uint64_t)e;
        keep.push_back(e);
      }
      keep.push_back((int32_t)p);
      h += (uint64_t)p;
      E[i].swap(keep);
      keep.clear();
      for (int32_t j : A[i])
        if (nv[j] > 0 && st[j] == VAR && mark[j] != stamp) {   // not p, not in L_p
          d += nv[j];
          h += (uint64_t)j;
          keep.push_back(j);
        }
      A[i].swap(keep);
      if (E[i].size() == 1 && A[i].empty()) {   // only neighbour is element p: eliminate with p
        nel += nv[i];
        degme -= nv[i];
        join(p, i);
        nv[i] = 0;
        st[i] = DEAD;
        std::vector<int32_t>().swap(E[i]);
        continue;
      }
      const int64_t lpi = degme - nv[i];
      deg[i] = std::min(deg[i] + lpi, d + lpi);
      hv.push_back({h * 1315423911ull + E[i].size() * 31 + A[i].size(), i});
    }
    // ---- supervariables: equal (E_i, A_i) among the survivors ----
    std::sort(hv.begin(), hv.end());
    for (size_t a = 0; a < hv.size(); ++a) {
      const int32_t i = hv[a].second;
      if (nv[i] == 0) continue;
      bool marked = false;
      for (size_t b = a + 1; b < hv.size() && hv[b].first == hv[a].first; ++b) {
        const int32_t j = hv[b].second;
        if (nv[j] == 0 || E[j].size() != E[i].size() || A[j].size() != A[i].size()) continue;
        if (!marked) {
          ++stamp2;
          for (int32_t e : E[i]) mark2[e] = stamp2;
          for (int32_t v : A[i]) mark2[v] = stamp2;
          marked = true;
        }
        bool same = true;
        for (int32_t e : E[j]) same = same && mark2[e] == stamp2;
        for (int32_t v : A[j]) same = same && mark2[v] == stamp2;
        if (!same) continue;
        nv[i] += nv[j];
        deg[i] -= nv[j];
        nv[j] = 0;
        st[j] = DEAD;
        join(i, j);
        std::vector<int32_t>().swap(E[j]);
        std::vector<int32_t>().swap(A[j]);
      }
    }
    // ---- finalize element p, reinsert its variables ----
    keep.clear();
    int64_t wp = 0;
    for (int32_t i : Lp)
      if (nv[i] > 0 && st[i] == VAR) {
        keep.push_back(i);
        wp += nv[i];
      }
    L[p].swap(keep);
    ew[p] = wp;
    for (int32_t i : L[p]) {
      deg[i] = std::max<int64_t>(0, std::min(deg[i], n - nel - nv[i]));
      ins(i);
      mindeg = std::min(mindeg, deg[i]);
    }
    for (int64_t v = p; v >= 0; v = gnext[v]) perm.push_back(v);
    wflg += n + 1;   // every w[e] set in this step is < the next wflg
  }
  return perm;
}

}  // namespace smlu
