// Dev probe: sustained v_mfma_f64_16x16x4_f64 issue rate with every CU busy, long enough
// (~50-100 ms per case) for the clock to settle.  The MFMAs are emitted by inline asm on
// accumulators pinned in architectural VGPRs ("+v"), so the loop body is exactly NACC
// back-to-back independent MFMAs (no AGPR copies, no other instructions); W workgroups of
// 256 threads per CU give W waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s\n", hipGetErrorString(e)); exit(1);} } while (0)

typedef double v4d __attribute__((ext_vector_type(4)));
#define MF(i) asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %2, %0" : "+v"(acc[i]) : "v"(a[(i) & 3]), "v"(b[((i) >> 2) & 3]))

template <int NACC>
__global__ __launch_bounds__(256, 2) void k_mfma(double* out, int iters) {
  v4d acc[16];
  double a[4], b[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    a[i] = 1.0 + 1e-3 * (threadIdx.x + i);
    b[i] = 1.0 - 1e-3 * (threadIdx.x + 3 * i);
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = (v4d){0.0, 0.0, 0.0, 0.0};
  for (int it = 0; it < iters; ++it) {
    MF(0); if (NACC > 1) MF(1); if (NACC > 2) MF(2); if (NACC > 3) MF(3);
    if (NACC > 4) { MF(4); MF(5); MF(6); MF(7); }
    if (NACC > 8) { MF(8); MF(9); MF(10); MF(11); MF(12); MF(13); MF(14); MF(15); }
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <class F>
void timeit(const char* name, F launch, double flops) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  launch(); CK(hipDeviceSynchronize());
  launch(); CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  launch();
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  printf("%-40s %.2f TF/s  (%.3f ms)\n", name, flops / ms / 1e9, ms);
}

int main() {
  double* out;
  CK(hipMalloc(&out, (size_t)256 * 8 * 256 * 8));
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, 0));
  const int ncu = p.multiProcessorCount;
  printf("CUs %d clock %d kHz\n", ncu, p.clockRate);
  for (int w = 1; w <= 2; ++w) {
    const int nwg = ncu * w;
    const int total = 640000 / w;   // MFMAs per wave
    char nm[80];
    for (int nacc : {1, 2, 4, 8, 16}) {
      snprintf(nm, sizeof nm, "mfma f64 asm, %2d acc, %d wave/SIMD", nacc, w);
      const int iters = total / nacc;
      const double fl = 2048.0 * nwg * 4.0 * iters * nacc;
      if (nacc == 1) timeit(nm, [&] { k_mfma<1><<<nwg, 256>>>(out, iters); }, fl);
      if (nacc == 2) timeit(nm, [&] { k_mfma<2><<<nwg, 256>>>(out, iters); }, fl);
      if (nacc == 4) timeit(nm, [&] { k_mfma<4><<<nwg, 256>>>(out, iters); }, fl);
      if (nacc == 8) timeit(nm, [&] { k_mfma<8><<<nwg, 256>>>(out, iters); }, fl);
      if (nacc == 16) timeit(nm, [&] { k_mfma<16><<<nwg, 256>>>(out, iters); }, fl);
    }
  }
  return 0;
}
