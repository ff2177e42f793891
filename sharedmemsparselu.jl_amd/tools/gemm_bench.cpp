// gemm_bench — dev microbenchmark of the fp64 Schur-update kernels (C -= A*B) in isolation:
// correctness of the 128-tile kernel against the 64-tile kernel, and TFLOP/s per shape.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../csrc/device.hpp"
namespace smlu { hipError_t launch_gemm(hipStream_t, int64_t, const GemmTask*, int, int, int64_t); }
using namespace smlu;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %s\n", hipGetErrorString(e), #x); exit(1);} } while (0)

static void fill(std::vector<double>& v, unsigned seed) { srand(seed); for (auto& x : v) x = rand() / (double)RAND_MAX - 0.5; }

int main(int argc, char** argv) {
  struct Shape { int m, n, k, lda = 0, ldb = 0, ldc = 0; } shapes[] = {{4096, 4096, 4096}, {8192, 8192, 1024}, {16384, 16384, 64}, {12000, 12000, 6000}, {1000, 1000, 300}, {300, 5000, 32}, {777, 1333, 129},
                                            {18000, 192, 64}, {192, 18000, 64}, {6000, 6000, 256}, {3000, 3000, 256}, {1500, 1500, 1000}, {18000, 256, 256}};
  std::vector<Shape> sv(std::begin(shapes), std::end(shapes));
  if (argc > 1) {   // shapes from the command line: m,n,k ...
    sv.clear();
    for (int a = 1; a < argc; ++a) {   // m,n,k or m,n,k,lda,ldb,ldc
      Shape x;
      if (sscanf(argv[a], "%d,%d,%d,%d,%d,%d", &x.m, &x.n, &x.k, &x.lda, &x.ldb, &x.ldc) >= 3) sv.push_back(x);
    }
  }
  // variants: tile codes of launch_gemm (GB_TILES="128,130"); the first one is the reference
  std::vector<int> tiles_list = {64, 128, 130};
  if (const char* e = std::getenv("GB_TILES")) {
    tiles_list.clear();
    for (const char* p = e; *p;) { tiles_list.push_back(std::atoi(p)); while (*p && *p != ',') ++p; if (*p) ++p; }
  }
  const int NV = (int)tiles_list.size();
  hipStream_t st; CK(hipStreamCreate(&st));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (auto sh : sv) {
    int m = sh.m, n = sh.n, k = sh.k, lda = sh.lda ? sh.lda : m + 3, ldb = sh.ldb ? sh.ldb : k + 1,
        ldc = sh.ldc ? sh.ldc : m + 5;
    std::vector<double> hA((size_t)lda * k), hB((size_t)ldb * n), hC((size_t)ldc * n);
    fill(hA, 1); fill(hB, 2); fill(hC, 3);
    double *A, *B, *C1, *C2; GemmTask* dt;
    CK(hipMalloc(&A, hA.size() * 8)); CK(hipMalloc(&B, hB.size() * 8)); CK(hipMalloc(&C1, hC.size() * 8)); CK(hipMalloc(&C2, hC.size() * 8));
    CK(hipMemcpy(A, hA.data(), hA.size() * 8, hipMemcpyHostToDevice)); CK(hipMemcpy(B, hB.data(), hB.size() * 8, hipMemcpyHostToDevice));
    CK(hipMalloc(&dt, sizeof(GemmTask)));
    std::vector<double> res(NV, 0.0), vdiff(NV, 0.0);
    std::vector<double> ref(hC.size());
    for (int variant = 0; variant < NV; ++variant) {
      int tile = tiles_list[variant];
      double* C = variant == 0 ? C1 : C2;
      GemmTask t{}; t.A = A; t.B = B; t.C = C; t.m = m; t.n = n; t.k = k; t.lda = lda; t.ldb = ldb; t.ldc = ldc;
      const int tsm = tile >= 128 ? 128 : 64, tsn = tsm;
      t.tiles_m = (m + tsm - 1) / tsm; t.tile0 = 0;
      int64_t tiles = (int64_t)t.tiles_m * ((n + tsn - 1) / tsn);
      CK(hipMemcpy(dt, &t, sizeof t, hipMemcpyHostToDevice));
      CK(hipMemcpy(C, hC.data(), hC.size() * 8, hipMemcpyHostToDevice));
      CK(launch_gemm(st, tiles, dt, 1, tile, 0));   // one correctness pass
      CK(hipStreamSynchronize(st));
      {
        std::vector<double> r(hC.size());
        CK(hipMemcpy(r.data(), C, r.size() * 8, hipMemcpyDeviceToHost));
        if (variant == 0) ref = r;
        else
          for (size_t o = 0; o < r.size(); ++o) vdiff[variant] = fmax(vdiff[variant], fabs(r[o] - ref[o]));
      }
      int reps = (double)m * n * k > 1e11 ? 3 : 20;
      CK(hipEventRecord(e0, st));
      for (int r = 0; r < reps; ++r) CK(launch_gemm(st, tiles, dt, 1, tile, 0));
      CK(hipEventRecord(e1, st)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      res[variant] = 2.0 * m * n * (double)k * reps / (ms * 1e-3) / 1e12;
    }
    printf("m=%6d n=%6d k=%6d ld=%d,%d,%d ", m, n, k, lda, ldb, ldc);
    for (int v = 0; v < NV; ++v) printf(" t%d %6.2f TF (maxdiff vs t%d %.1e)", tiles_list[v], res[v], tiles_list[0], vdiff[v]);
    printf("\n");
    CK(hipFree(A)); CK(hipFree(B)); CK(hipFree(C1)); CK(hipFree(C2)); CK(hipFree(dt));
  }
  return 0;
}
