// clock_probe — effective shader clock of a lone workgroup vs a full-chip launch
// (delta s_memtime / delta s_memrealtime * 100 MHz), and latency of a dependent fp64 chain.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
__global__ void probe(unsigned long long* out, int iters, double* sink) {
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  double x = threadIdx.x * 1e-3, y = 1.0000001;
  for (int i = 0; i < iters; ++i) x = fma(x, y, 1e-9);
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) { out[2 * blockIdx.x] = t1 - t0; out[2 * blockIdx.x + 1] = r1 - r0; }
  if (x == 12345.0) sink[0] = x;
}
int main() {
  unsigned long long* d; double* sink;
  hipMalloc(&d, sizeof(unsigned long long) * 2 * 4096); hipMalloc(&sink, 8);
  for (int blocks : {1, 8, 256, 2048}) {
    for (int rep = 0; rep < 3; ++rep) {
      hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
      hipEventRecord(a);
      probe<<<blocks, 256>>>(d, 200000, sink);
      hipEventRecord(b); hipEventSynchronize(b);
      float ms; hipEventElapsedTime(&ms, a, b);
      std::vector<unsigned long long> h(2 * blocks);
      hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost);
      double mt = h[0], rt = h[1];
      printf("blocks %5d rep %d: wall %.3f ms, clock %.0f MHz, cycles/dep-fma %.2f\n", blocks, rep, ms,
             mt / rt * 100.0, mt / 200000.0);
    }
  }
  return 0;
}
