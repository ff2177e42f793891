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

// fp64 MFMA (v_mfma_f64_16x16x4_f64): NACC independent 16x16 accumulators per wave
typedef double v4d __attribute__((ext_vector_type(4)));
template <int NACC>
__global__ __launch_bounds__(256) void k_mfma(double* out, int iters) {
  v4d acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) acc[i] = (v4d){0.0, 0.0, 0.0, 0.0};
  double a = 1.0 + 1e-3 * threadIdx.x, b = 1.0 - 1e-3 * threadIdx.x;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

// Mixed issue: even waves run MFMA chains, odd waves run VALU FMA chains on the same SIMDs
// (does the fp64 matrix pipe overlap the fp64 VALU?).  flops counted per wave kind.
__global__ __launch_bounds__(256) void k_mixed(double* out, int iters_m, int iters_v) {
  const int wv = threadIdx.x >> 6;
  double s = 0;
  if (wv & 1) {
    double acc[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) acc[i] = threadIdx.x + i;
    const double a = 0.999, b = 1e-3;
    for (int it = 0; it < iters_v; ++it) {
#pragma unroll
      for (int i = 0; i < 32; ++i) acc[i] = fma(acc[i], a, b);
    }
#pragma unroll
    for (int i = 0; i < 32; ++i) s += acc[i];
  } else {
    v4d acc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = (v4d){0.0, 0.0, 0.0, 0.0};
    double a = 1.0 + 1e-3 * threadIdx.x, b = 1.0 - 1e-3 * threadIdx.x;
    for (int it = 0; it < iters_m; ++it) {
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  }
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
  for (int w = 1; w <= 2; ++w) {
    const int nwg = 256 * w;
    char nm[64];
    snprintf(nm, sizeof nm, "mfma f64 16x16x4, 8 acc, %d WG/CU", w);
    // flops per MFMA = 2*16*16*4 = 2048, per wave; 4 waves per WG
    timeit(nm, [&] { k_mfma<8><<<nwg, 256>>>(out, iters / 8); }, 2048.0 * nwg * 4.0 * (iters / 8) * 8);
    snprintf(nm, sizeof nm, "mfma f64 16x16x4, 16 acc, %d WG/CU", w);
    timeit(nm, [&] { k_mfma<16><<<nwg, 256>>>(out, iters / 16); }, 2048.0 * nwg * 4.0 * (iters / 16) * 16);
  }
  {
    // per MFMA wave: iters_m*8 MFMAs * 2048 flops; per VALU wave: iters_v*32 FMAs * 64 lanes * 2
    const int nwg = 512, im = iters / 8, iv = iters / 4;
    const double fm = 2048.0 * im * 8, fv = 128.0 * iv * 32;
    timeit("mixed mfma+valu waves, 2 WG/CU", [&] { k_mixed<<<nwg, 256>>>(out, im, iv); }, nwg * 2.0 * (fm + fv));
    timeit("mixed: mfma waves only", [&] { k_mixed<<<nwg, 256>>>(out, im, 0); }, nwg * 2.0 * fm);
    timeit("mixed: valu waves only", [&] { k_mixed<<<nwg, 256>>>(out, 0, iv); }, nwg * 2.0 * fv);
  }
  return 0;
}
