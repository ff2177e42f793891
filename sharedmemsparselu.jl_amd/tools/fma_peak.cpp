// Dev probe: sustained fp64 VALU FMA throughput with every CU busy (no memory traffic), with
// one operand uniform (SGPR) and with all three operands in VGPRs (the GEMM micro-kernel shape:
// 8x8 outer product per k, a[8] and b[8] in registers).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s\n", hipGetErrorString(e)); exit(1);} } while (0)

template <int NACC>
__global__ __launch_bounds__(256) void k_fma_s(double* out, int iters, double a, double b) {
  double acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) acc[i] = threadIdx.x + i;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = fma(acc[i], a, b);
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < NACC; ++i) s += acc[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

// 8x8 outer product per iteration, a/b perturbed each iteration so they stay in VGPRs
__global__ __launch_bounds__(256, 2) void k_fma_outer(double* out, int iters, double da) {
  double acc[8][8], a[8], b[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    a[i] = 1.0 + 1e-3 * (threadIdx.x + i);
    b[i] = 1.0 - 1e-3 * (threadIdx.x + 2 * i);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = 0.0;
  }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = fma(a[i], b[j], acc[i][j]);
    a[it & 7] += da;   // keep a live and varying (1 extra add per 64 FMAs)
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) s += acc[i][j];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <class F>
void timeit(const char* name, F launch, double flops) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  launch(); CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  launch();
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  printf("%-34s %.2f TF/s  (%.3f ms)\n", name, flops / ms / 1e9, ms);
}

int main() {
  double* out;
  CK(hipMalloc(&out, (size_t)256 * 4 * 256 * 8));
  const int iters = 20000;
  for (int w = 1; w <= 2; ++w) {
    const int nwg = 256 * w;
    char nm[64];
    snprintf(nm, sizeof nm, "sgpr operand, 64 acc, %d WG/CU", w);
    timeit(nm, [&] { k_fma_s<64><<<nwg, 256>>>(out, iters, 0.999, 1e-3); }, 2.0 * nwg * 256.0 * iters * 64);
    snprintf(nm, sizeof nm, "vgpr 8x8 outer product, %d WG/CU", w);
    timeit(nm, [&] { k_fma_outer<<<nwg, 256>>>(out, iters / 4, 1e-9); }, 2.0 * nwg * 256.0 * (iters / 4) * 64);
  }
  return 0;
}
