// Dev probe: rocBLAS dgemm (C -= A*B, deterministic: atomics not allowed) against the library's
// MFMA tile (launch_gemm tile 129) on the refactor's GEMM shapes: TFLOP/s and max relative
// difference of the results; and run-to-run bitwise determinism of rocBLAS.
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../csrc/device.hpp"
namespace smlu { hipError_t launch_gemm(hipStream_t, int64_t, const GemmTask*, int, int, int64_t); }
using namespace smlu;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %s\n", hipGetErrorString(e), #x); exit(1);} } while (0)
#define RB(x) do { rocblas_status s = (x); if (s != rocblas_status_success) { printf("rocblas %d at %s\n", (int)s, #x); exit(1);} } while (0)

static void fill(std::vector<double>& v, unsigned seed) { srand(seed); for (auto& x : v) x = rand() / (double)RAND_MAX - 0.5; }

int main(int argc, char** argv) {
  struct Shape { int m, n, k; };
  std::vector<Shape> sv = {{8192, 8192, 8192}, {16000, 16000, 384}, {16000, 16000, 1536}, {12000, 12000, 3700},
                           {9000, 9000, 2300}, {3000, 3000, 256}, {18000, 384, 384}, {1000, 1000, 300}};
  if (argc > 1) {
    sv.clear();
    for (int a = 1; a < argc; ++a) { Shape x; if (sscanf(argv[a], "%d,%d,%d", &x.m, &x.n, &x.k) == 3) sv.push_back(x); }
  }
  hipStream_t st; CK(hipStreamCreate(&st));
  rocblas_handle hb; RB(rocblas_create_handle(&hb)); RB(rocblas_set_stream(hb, st));
  RB(rocblas_set_atomics_mode(hb, rocblas_atomics_not_allowed));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (auto sh : sv) {
    int m = sh.m, n = sh.n, k = sh.k, lda = m + 3, ldb = k + 1, ldc = m + 5;
    std::vector<double> hA((size_t)lda * k), hB((size_t)ldb * n), hC((size_t)ldc * n);
    fill(hA, 1); fill(hB, 2); fill(hC, 3);
    double *A, *B, *C1, *C2, *C3; GemmTask* dt;
    CK(hipMalloc(&A, hA.size() * 8)); CK(hipMalloc(&B, hB.size() * 8));
    CK(hipMalloc(&C1, hC.size() * 8)); CK(hipMalloc(&C2, hC.size() * 8)); CK(hipMalloc(&C3, hC.size() * 8));
    CK(hipMemcpy(A, hA.data(), hA.size() * 8, hipMemcpyHostToDevice)); CK(hipMemcpy(B, hB.data(), hB.size() * 8, hipMemcpyHostToDevice));
    CK(hipMalloc(&dt, sizeof(GemmTask)));
    GemmTask t{}; t.A = A; t.B = B; t.C = C1; t.m = m; t.n = n; t.k = k; t.lda = lda; t.ldb = ldb; t.ldc = ldc;
    t.tiles_m = (m + 127) / 128; t.tile0 = 0;
    int64_t tiles = (int64_t)t.tiles_m * ((n + 127) / 128);
    CK(hipMemcpy(dt, &t, sizeof t, hipMemcpyHostToDevice));
    const double alpha = -1.0, beta = 1.0;
    auto ours = [&](double* C) { (void)C; CK(launch_gemm(st, tiles, dt, 1, 130, 0)); };
    auto vend = [&](double* C) {
      RB(rocblas_dgemm(hb, rocblas_operation_none, rocblas_operation_none, m, n, k, &alpha, A, lda, B, ldb, &beta, C, ldc));
    };
    CK(hipMemcpy(C1, hC.data(), hC.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(C2, hC.data(), hC.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(C3, hC.data(), hC.size() * 8, hipMemcpyHostToDevice));
    ours(C1); vend(C2); vend(C3);
    CK(hipStreamSynchronize(st));
    std::vector<double> r1(hC.size()), r2(hC.size()), r3(hC.size());
    CK(hipMemcpy(r1.data(), C1, r1.size() * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(r2.data(), C2, r2.size() * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(r3.data(), C3, r3.size() * 8, hipMemcpyDeviceToHost));
    double md = 0, mx = 0; bool same = true;
    for (int j = 0; j < n; ++j) for (int i = 0; i < m; ++i) {
      size_t o = (size_t)j * ldc + i;
      md = fmax(md, fabs(r1[o] - r2[o])); mx = fmax(mx, fabs(r1[o]));
      if (r2[o] != r3[o]) same = false;
    }
    double tf[2];
    for (int v = 0; v < 2; ++v) {
      int reps = (double)m * n * k > 1e11 ? 3 : 20;
      CK(hipEventRecord(e0, st));
      for (int r = 0; r < reps; ++r) { if (v == 0) ours(C1); else vend(C2); }
      CK(hipEventRecord(e1, st)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      tf[v] = 2.0 * m * n * (double)k * reps / (ms * 1e-3) / 1e12;
    }
    printf("m=%6d n=%6d k=%6d  ours %6.2f TF  rocblas %6.2f TF  rel diff %.1e  rocblas repeat bitwise %s\n",
           m, n, k, tf[0], tf[1], md / mx, same ? "yes" : "NO");
    CK(hipFree(A)); CK(hipFree(B)); CK(hipFree(C1)); CK(hipFree(C2)); CK(hipFree(C3)); CK(hipFree(dt));
  }
  return 0;
}
