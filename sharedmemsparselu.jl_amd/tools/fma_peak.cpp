// Dev probe: sustained fp64 VALU FMA throughput with every CU busy (no memory traffic).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s\n", hipGetErrorString(e)); exit(1);} } while (0)

template <int NACC>
__global__ __launch_bounds__(256) void k_fma(double* out, int iters, double a, double b) {
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

template <int NACC>
void run(int wgs_per_cu) {
  const int nwg = 256 * wgs_per_cu, iters = 20000;
  double* out;
  CK(hipMalloc(&out, (size_t)nwg * 256 * 8));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  k_fma<NACC><<<nwg, 256>>>(out, 10, 0.999, 1e-3);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  k_fma<NACC><<<nwg, 256>>>(out, iters, 0.999, 1e-3);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  double fl = 2.0 * nwg * 256.0 * iters * NACC;
  printf("NACC=%d wg/cu=%d  %.2f TF/s  (%.3f ms)\n", NACC, wgs_per_cu, fl / ms / 1e9, ms);
  CK(hipFree(out));
}

int main() {
  run<8>(1); run<8>(2); run<16>(1); run<16>(2); run<32>(1); run<32>(2); run<64>(1); run<64>(2);
  return 0;
}
