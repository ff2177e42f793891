// trsm_bench — dev microbenchmark of the blocked-front triangular-solve kernels on one dense
// synthetic front (ns = 4096, nu = 8192, panel width 64): the outer-phase U-row solve
// (k_trsm_u, 12k columns) and the per-step solve (k_step_trsm), generic vs full-width paths.
// Checks that both paths give bitwise-identical results.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "../csrc/device.hpp"
namespace smlu {
hipError_t launch_step_trsm(hipStream_t, int, const FrontTile*, int, int64_t, const FrontTile*, int, int64_t,
                            int, int, const SNode*, double*, double*, int32_t*, double*, double);
hipError_t launch_trsm_u(hipStream_t, int64_t, const FrontTile*, int, int, int, const SNode*, double*,
                         double*, const int32_t*, int64_t);
hipError_t launch_panel1(hipStream_t, int, int, int, int, int, const int32_t*, const SNode*, double*, double*,
                         int32_t*, int32_t*, int64_t, int32_t*, double*, double);
}
using namespace smlu;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %s\n", hipGetErrorString(e), #x); exit(1);} } while (0)

int main() {
  const int ns = 4096, nu = 8192, nb = 64, OB = 256;
  const int64_t M = ns + nu;
  const size_t nL = (size_t)M * ns, nU = (size_t)ns * nu;
  std::vector<double> h(nL + nU);
  srand(7);
  for (auto& v : h) v = (rand() / (double)RAND_MAX - 0.5) * 0.05;
  for (int j = 0; j < ns; ++j) h[(size_t)j * M + j] = 1.0 + (j % 7);   // well-conditioned triangles
  double *d0, *d1, *sc, *growth; int32_t* info;
  CK(hipMalloc(&d0, h.size() * 8)); CK(hipMalloc(&d1, h.size() * 8)); CK(hipMalloc(&sc, 8));
  CK(hipMalloc(&growth, 8)); CK(hipMalloc(&info, 4));
  SNode s{}; s.first = 0; s.Loff = 0; s.Uoff = nL; s.Foff = -1; s.ns = ns; s.nu = nu; s.nb = nb; s.mode = 2;
  s.parent = -1;
  SNode* dsn; CK(hipMalloc(&dsn, sizeof s)); CK(hipMemcpy(dsn, &s, sizeof s, hipMemcpyHostToDevice));
  hipStream_t st; CK(hipStreamCreate(&st));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto timeit = [&](auto fn, int reps) {
    fn(); CK(hipStreamSynchronize(st));
    CK(hipEventRecord(e0, st));
    for (int r = 0; r < reps; ++r) fn();
    CK(hipEventRecord(e1, st)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    return ms * 1e3 / reps;
  };
  if (std::getenv("PANEL_ONLY")) goto panel;
  {
  // outer phase: sub-panel at kb = 0 of the block [0, 256): columns [256, M)
  FrontTile ft{0, 0, 0};
  FrontTile* dft; CK(hipMalloc(&dft, sizeof(FrontTile) * 2));
  CK(hipMemcpy(dft, &ft, sizeof ft, hipMemcpyHostToDevice));
  const int64_t nwg_u = (M - OB + 255) / 256;
  double t_u[2];
  std::vector<double> r[2];
  for (int fast = 0; fast < 2; ++fast) {
    double* d = fast ? d1 : d0;
    CK(hipMemcpy(d, h.data(), h.size() * 8, hipMemcpyHostToDevice));
    CK(launch_trsm_u(st, nwg_u, dft, 1, OB, 1 | (fast << 1), dsn, d, sc, nullptr, 0));
    CK(hipStreamSynchronize(st));
    r[fast].resize(h.size());
    CK(hipMemcpy(r[fast].data(), d, h.size() * 8, hipMemcpyDeviceToHost));
    t_u[fast] = timeit([&] { (void)launch_trsm_u(st, nwg_u, dft, 1, OB, 1 | (fast << 1), dsn, d, sc, nullptr, 0); }, 20);
  }
  printf("trsm_u  (64 x %lld columns, %lld WGs): generic %7.1f us  fast %7.1f us  bitwise %s\n",
         (long long)(M - OB), (long long)nwg_u, t_u[0], t_u[1],
         memcmp(r[0].data(), r[1].data(), h.size() * 8) == 0 ? "equal" : "DIFFERENT");
  // step solve at kb = 0: U role columns [64, 256) (1 WG), L role rows [64, M)
  FrontTile fts[2] = {{0, 0, 0}, {0, 0, 0}};
  CK(hipMemcpy(dft, fts, sizeof fts, hipMemcpyHostToDevice));
  const int64_t nUw = 1, nLw = (M - nb + 255) / 256;
  double t_s[2];
  for (int fast = 0; fast < 2; ++fast) {
    double* d = fast ? d1 : d0;
    CK(hipMemcpy(d, h.data(), h.size() * 8, hipMemcpyHostToDevice));
    CK(launch_step_trsm(st, 64, dft, 1, nUw, dft + 1, 1, nLw, 0, OB, dsn, d, sc, info, growth, 0.1));
    CK(hipStreamSynchronize(st));
    CK(hipMemcpy(r[fast].data(), d, h.size() * 8, hipMemcpyDeviceToHost));
    t_s[fast] = timeit([&] { (void)launch_step_trsm(st, 64, dft, 1, nUw, dft + 1, 1, nLw, 0, OB, dsn, d, sc, info, growth, 0.1); }, 20);
  }
  printf("step_trsm (U 192 cols + L %lld rows, %lld WGs): generic %7.1f us  fast %7.1f us  bitwise %s\n",
         (long long)(M - nb), (long long)(nUw + nLw), t_s[0], t_s[1],
         memcmp(r[0].data(), r[1].data(), h.size() * 8) == 0 ? "equal" : "DIFFERENT");
  }
panel:
  // panel at kb = 0 (64 x 64 diagonal tile, diagonal preference 0.1)
  {
    int32_t* dl; int32_t* rp; int32_t* sw;
    CK(hipMalloc(&dl, 8)); CK(hipMalloc(&rp, 4 * ns)); CK(hipMalloc(&sw, 4 * 256));
    int32_t hl[2] = {0, 0};
    CK(hipMemcpy(dl, hl, 8, hipMemcpyHostToDevice));
    CK(hipMemset(rp, 0, 4 * ns));
    CK(hipMemcpy(d0, h.data(), h.size() * 8, hipMemcpyHostToDevice));
    CK(launch_panel1(st, 1, 0, 64, 64, 0, dl, dsn, d0, sc, rp, sw, 129, info, growth, 0.1));
    CK(hipStreamSynchronize(st));
    std::vector<double> p1((size_t)M * 64);
    CK(hipMemcpy(p1.data(), d0, p1.size() * 8, hipMemcpyDeviceToHost));
    double cs = 0;
    for (int j = 0; j < 64; ++j) for (int i = 0; i < 64; ++i) cs += p1[(size_t)j * M + i] * (1 + i + 64 * j);
    {  // pivoting case: a tile without diagonal dominance
      std::vector<double> h2(h.begin(), h.begin() + (size_t)M * 64);
      for (int j = 0; j < 64; ++j) for (int i = 0; i < 64; ++i) h2[(size_t)j * M + i] = (rand() / (double)RAND_MAX - 0.5);
      // host reference: threshold partial pivoting with diagonal preference (tol 0.1), LAPACK swaps
      std::vector<double> ref(64 * 64);
      for (int j = 0; j < 64; ++j) for (int i = 0; i < 64; ++i) ref[j * 64 + i] = h2[(size_t)j * M + i];
      int nswap = 0;
      for (int k = 0; k < 64; ++k) {
        double akk = ref[k * 64 + k];
        bool beats = false;
        for (int i = k + 1; i < 64; ++i) if (fabs(ref[k * 64 + i]) * 0.1 > fabs(akk)) beats = true;
        int pr = k;
        if (beats || akk == 0.0) {
          double am = -1; for (int i = k; i < 64; ++i) if (fabs(ref[k * 64 + i]) > am) { am = fabs(ref[k * 64 + i]); pr = i; }
        }
        if (pr != k) { ++nswap; for (int j = 0; j < 64; ++j) std::swap(ref[j * 64 + k], ref[j * 64 + pr]); }
        for (int i = k + 1; i < 64; ++i) {
          double l = ref[k * 64 + i] / ref[k * 64 + k];
          ref[k * 64 + i] = l;
          for (int j = k + 1; j < 64; ++j) ref[j * 64 + i] = fma(-l, ref[j * 64 + k], ref[j * 64 + i]);
        }
      }
      CK(hipMemcpy(d1, h2.data(), h2.size() * 8, hipMemcpyHostToDevice));
      CK(launch_panel1(st, 1, 0, 64, 64, 0, dl, dsn, d1, sc, rp, sw, 129, info, growth, 0.1));
      CK(hipStreamSynchronize(st));
      CK(hipMemcpy(h2.data(), d1, h2.size() * 8, hipMemcpyDeviceToHost));
      double cs2 = 0;
      for (int j = 0; j < 64; ++j) for (int i = 0; i < 64; ++i) cs2 += h2[(size_t)j * M + i] * (1 + i + 64 * j);
      std::vector<int32_t> hs(256);
      CK(hipMemcpy(hs.data(), sw, 4 * 256, hipMemcpyDeviceToHost));
      double md = 0; int bad = -1;
      for (int j = 0; j < 64; ++j) for (int i = 0; i < 64; ++i) {
        double d = fabs(h2[(size_t)j * M + i] - ref[j * 64 + i]) / (1 + fabs(ref[j * 64 + i]));
        if (d > md) { md = d; if (d > 1e-10 && bad < 0) bad = j * 64 + i; }
      }
      printf("pivoting tile: checksum %.17g  moved rows %d  host transpositions %d  max rel diff vs host %.2e (first bad col %d row %d)\n",
             cs2, hs[0], nswap, md, bad < 0 ? -1 : bad / 64, bad < 0 ? -1 : bad % 64);
    }
    double tp = timeit([&] { (void)launch_panel1(st, 1, 0, 64, 64, 0, dl, dsn, d0, sc, rp, sw, 129, info, growth, 0.1); }, 20);
    printf("panel_reg<64,1> (64 x 64 tile): %7.1f us   checksum %.17g\n", tp, cs);
  }
  return 0;
}
