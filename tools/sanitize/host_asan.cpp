// Host AddressSanitizer / UBSan driver (SURVEY §5 "race detection / sanitizers": host side).
// Builds the host symbolic plan (csrc/plan.cpp, ordering.cpp, amd.cpp) for several inputs and
// every ordering, the multi-GPU partition, per-rank layouts and the projection, and runs the CPU
// oracle (oracle/oracle.c fixed-pivot LU + solves, oracle/mf.c multifrontal pivot-choosing LU) on
// the plan's assembly tree -- all under -fsanitize=address,undefined (tools/sanitize/Makefile).
// No GPU code is compiled: device kernels cannot run under the sanitizers on this pool.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <vector>

#include "../../oracle/oracle.h"
#include "../../sharedmemsparselu.jl_amd/csrc/plan.hpp"

using namespace smlu;

struct Csc {
  int64_t n = 0;
  std::vector<int64_t> cp, ri;
  std::vector<double> v;
};

static Csc from_triplets(int64_t n, std::vector<std::vector<std::pair<int64_t, double>>>& cols) {
  Csc A;
  A.n = n;
  A.cp.push_back(0);
  for (int64_t j = 0; j < n; ++j) {
    auto& c = cols[j];
    std::sort(c.begin(), c.end());
    for (size_t k = 0; k < c.size(); ++k) {
      if (k > 0 && c[k].first == c[k - 1].first) { A.v.back() += c[k].second; continue; }
      A.ri.push_back(c[k].first);
      A.v.push_back(c[k].second);
    }
    A.cp.push_back((int64_t)A.ri.size());
  }
  return A;
}

static Csc poisson3d(int64_t m) {
  const int64_t n = m * m * m;
  std::vector<std::vector<std::pair<int64_t, double>>> cols(n);
  for (int64_t k = 0; k < m; ++k)
    for (int64_t j = 0; j < m; ++j)
      for (int64_t i = 0; i < m; ++i) {
        const int64_t v = i + m * (j + m * k);
        cols[v].push_back({v, 6.0});
        const int64_t nb[6][3] = {{i - 1, j, k}, {i + 1, j, k}, {i, j - 1, k}, {i, j + 1, k}, {i, j, k - 1}, {i, j, k + 1}};
        for (auto& t : nb)
          if (t[0] >= 0 && t[0] < m && t[1] >= 0 && t[1] < m && t[2] >= 0 && t[2] < m)
            cols[v].push_back({t[0] + m * (t[1] + m * t[2]), -1.0});
      }
  return from_triplets(n, cols);
}

static Csc random_sparse(int64_t n, double dens, bool dominant, unsigned seed) {
  std::mt19937_64 g(seed);
  std::uniform_real_distribution<double> u(0.0, 1.0);
  std::vector<std::vector<std::pair<int64_t, double>>> cols(n);
  std::vector<double> rowsum(n, 0.0);
  for (int64_t j = 0; j < n; ++j)
    for (int64_t i = 0; i < n; ++i)
      if (i != j && u(g) < dens) {
        const double x = u(g);
        cols[j].push_back({i, x});
        rowsum[i] += x;
      }
  for (int64_t j = 0; j < n; ++j) cols[j].push_back({j, dominant ? 1.0 + rowsum[j] : 1e-3 * u(g)});
  return from_triplets(n, cols);
}

static int check(bool ok, const char* what) {
  if (!ok) std::fprintf(stderr, "FAIL: %s\n", what);
  return ok ? 0 : 1;
}

static int run_case(const char* name, const Csc& A, int ordering, const int64_t* grid, bool dominant = true) {
  int bad = 0;
  PlanOptions o;
  o.ordering = ordering;
  if (grid)
    for (int d = 0; d < 3; ++d) o.grid[d] = grid[d];
  std::vector<int64_t> match;
  {
    std::vector<int32_t> r32(A.ri.begin(), A.ri.end());
    match = zero_free_diagonal(A.n, A.cp.data(), r32.data(), A.v.data());
  }
  Plan P;
  const std::string e = P.build(A.n, A.cp.data(), A.ri.data(), 0, o, nullptr, nullptr,
                                match.empty() ? nullptr : match.data());
  if (!e.empty()) {
    std::fprintf(stderr, "%s: plan failed: %s\n", name, e.c_str());
    return 1;
  }
  for (int np : {1, 2, 3, 8}) {
    P.compute_owners(np, 384);
    double t1 = 0;
    const double t = project_partition(P, 50.0, 100.0, 20.0, &t1);
    bad += check(t >= 0 && t1 >= 0 && std::isfinite(t), "projection finite");
    for (int r = 0; r < np; ++r) {
      RankLayout L;
      rank_layout(P, r, L);
      bad += check(L.store_size >= 0 && L.scratch_size >= 0, "rank layout sizes");
    }
  }
  // oracle: multifrontal pivot-choosing LU on the plan's tree, then the fixed-pivot LU with its p
  std::vector<int64_t> first(P.s_first.begin(), P.s_first.end()), parent(P.s_parent.begin(), P.s_parent.end()),
      rowptr(P.s_rowptr.begin(), P.s_rowptr.end()), rows(P.s_rows.begin(), P.s_rows.end());
  for (int mode : {1, 2}) {
    std::vector<int32_t> modes(P.nsup, mode);
    int st = 0;
    oracle_mf* mf = oracle_mf_create(A.n, A.cp.data(), A.ri.data(), P.p0.data(), P.q.data(), P.nsup, first.data(),
                                     parent.data(), rowptr.data(), rows.data(), modes.data(), 0.001, 0.1, 2, &st);
    bad += check(mf != nullptr, "oracle_mf_create");
    if (!mf) continue;
    const int fs = oracle_mf_factor(mf, A.v.data());
    std::vector<int32_t> rowperm(A.n), flags(P.nsup);
    std::vector<double> Rs(A.n);
    oracle_mf_result(mf, rowperm.data(), flags.data(), Rs.data());
    oracle_mf_destroy(mf);
    if (fs != 0) continue;   // singular under this candidate mode: nothing to solve
    std::vector<int64_t> p(A.n);
    for (int64_t s = 0; s < P.nsup; ++s)
      for (int64_t k = P.s_first[s]; k < P.s_first[s + 1]; ++k) p[k] = P.p0[P.s_first[s] + rowperm[k]];
    int st2 = 0;
    oracle_lu* F = oracle_lu_fixed(A.n, A.cp.data(), A.ri.data(), A.v.data(), Rs.data(), p.data(), P.q.data(), &st2);
    bad += check(F != nullptr, "oracle_lu_fixed");
    if (!F) continue;
    std::vector<double> b(A.n), x(A.n), r(A.n, 0.0);
    for (int64_t i = 0; i < A.n; ++i) b[i] = 1.0 + (double)(i % 7);
    oracle_ldiv(F, Rs.data(), p.data(), P.q.data(), b.data(), x.data());
    for (int64_t j = 0; j < A.n; ++j)
      for (int64_t k = A.cp[j]; k < A.cp[j + 1]; ++k) r[A.ri[k]] += A.v[k] * x[j];
    double rn = 0, bn = 0;
    for (int64_t i = 0; i < A.n; ++i) { rn = std::max(rn, std::fabs(r[i] - b[i])); bn = std::max(bn, std::fabs(b[i])); }
    bad += check(std::isfinite(rn) && (!dominant || rn <= 1e-10 * bn), "oracle solve residual");
    oracle_lu_free(F);
  }
  std::printf("%-28s n=%-6lld nsup=%-6lld ok=%d\n", name, (long long)A.n, (long long)P.nsup, bad == 0);
  return bad;
}

int main() {
  int bad = 0;
  const int64_t g12[3] = {12, 12, 12};
  const Csc P12 = poisson3d(12);
  bad += run_case("poisson3d_12 graph-nd", P12, 3, nullptr);
  bad += run_case("poisson3d_12 geometric-nd", P12, 2, g12);
  bad += run_case("poisson3d_12 amd", P12, 5, nullptr);
  bad += run_case("poisson3d_12 natural", P12, 1, nullptr);
  bad += run_case("random_dominant_800", random_sparse(800, 0.01, true, 47), 0, nullptr);
  bad += run_case("random_small_diag_300", random_sparse(300, 0.03, false, 5), 0, nullptr, false);
  bad += run_case("poisson3d_3", poisson3d(3), 0, nullptr);
  bad += run_case("one_entry", random_sparse(1, 0.0, true, 1), 0, nullptr);
  std::printf(bad == 0 ? "HOST SANITIZER RUN OK\n" : "HOST SANITIZER RUN FAILED\n");
  return bad == 0 ? 0 : 1;
}
