// Dev probe: sustained v_mfma_f64_16x16x4_f64 throughput with every CU busy, long enough
// (~50-100 ms per case) for the clock to settle: NACC independent accumulators per wave,
// W workgroups of 256 threads per CU, operands distinct per accumulator.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s\n", hipGetErrorString(e)); exit(1);} } while (0)

typedef double v4d __attribute__((ext_vector_type(4)));
template <int NACC>
__global__ __launch_bounds__(256) void k_mfma(double* out, int iters) {
  v4d acc[NACC];
  double a[4], b[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    a[i] = 1.0 + 1e-3 * (threadIdx.x + i);
    b[i] = 1.0 - 1e-3 * (threadIdx.x + 3 * i);
  }
#pragma unroll
  for (int i = 0; i < NACC; ++i) acc[i] = (v4d){0.0, 0.0, 0.0, 0.0};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i)
      acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[i & 3], b[(i >> 2) & 3], acc[i], 0, 0, 0);
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
  for (int w = 1; w <= 4; w *= 2) {
    const int nwg = ncu * w;
    const int iters = 40000 / w;
    char nm[80];
    snprintf(nm, sizeof nm, "mfma f64, 4 acc, %d WG/CU", w);
    timeit(nm, [&] { k_mfma<4><<<nwg, 256>>>(out, iters * 4); }, 2048.0 * nwg * 4.0 * iters * 16);
    snprintf(nm, sizeof nm, "mfma f64, 8 acc, %d WG/CU", w);
    timeit(nm, [&] { k_mfma<8><<<nwg, 256>>>(out, iters * 2); }, 2048.0 * nwg * 4.0 * iters * 16);
    snprintf(nm, sizeof nm, "mfma f64, 16 acc, %d WG/CU", w);
    timeit(nm, [&] { k_mfma<16><<<nwg, 256>>>(out, iters); }, 2048.0 * nwg * 4.0 * iters * 16);
  }
  return 0;
}
