// kernels_common.hpp — device helpers shared by the gfx950 kernel translation units
// (kernels_front.hip, kernels_gemm.hip, kernels_solve.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>

#include "device.hpp"

namespace smlu {

#define WAVE 64

__device__ __forceinline__ double wave_max_idx(double v, int& idx) {
  // max |.| with smallest index on ties; 64-lane butterfly
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    double ov = __shfl_xor(v, o, 64);
    int oi = __shfl_xor(idx, o, 64);
    if (ov > v || (ov == v && oi < idx)) { v = ov; idx = oi; }
  }
  return v;
}

// 1/x with one Newton step on the hardware estimate (v_rcp_f64): ~3 dependent fp64 ops instead
// of the ~10 of an IEEE division (a dependent fp64 op costs ~32 cycles on gfx950).  Used on the
// sequential pivot and triangular-solve chains; results stay within a few ulp of division.
__device__ __forceinline__ double recip(double x) {
  double r = __builtin_amdgcn_rcp(x);
  const double e = fma(-x, r, 1.0);
  r = fma(r, e, r);
  const double e2 = fma(-x, r, 1.0);
  return fma(r, e2, r);
}

// Global-address-space views of plain pointers: loads through them compile to global_load
// (vmcnt only) instead of flat_load, which also counts against lgkmcnt and so makes every LDS
// wait inside a loop wait for the global prefetch as well.
typedef __attribute__((address_space(1))) double gdbl;
template <typename T>
__device__ __forceinline__ __attribute__((address_space(1))) T* gbl(T* p) {
  return (__attribute__((address_space(1))) T*)p;
}

__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
  return v;
}

__device__ __forceinline__ void atomic_max_pos(double* addr, double v) {
  // v >= 0: IEEE ordering of non-negative doubles matches their bit patterns as u64.  The
  // stored maximum is read first and the atomic skipped when it already covers v: every front
  // reports into the same word, and same-address atomics serialise in L2 (they made the
  // hundred-thousand-front small-front levels atomic-bound).  The maximum only grows, so a
  // stale read costs at most one unneeded atomic.
  unsigned long long* p = reinterpret_cast<unsigned long long*>(addr);
  const unsigned long long b = (unsigned long long)__double_as_longlong(v);
  if (b <= __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
  atomicMax(p, b);
}

// info word per front: bit0 zero pivot, bit1 weak pivot, bits 2.. = 1 + first zero-pivot column
__device__ __forceinline__ void publish_info(int32_t* info, int flag, int errcol) {
  int v = *info | flag;
  if (errcol >= 0 && (v >> 2) == 0) v |= (errcol + 1) << 2;
  *info = v;
}

struct FrontPtrs {
  gdbl* L;
  gdbl* U;
  gdbl* F;
  int64_t M, ns, nu;
};

__device__ __forceinline__ FrontPtrs front_ptrs(const SNode& s, double* store, double* scratch) {
  FrontPtrs f;
  f.ns = s.ns;
  f.nu = s.nu;
  f.M = (int64_t)s.ns + s.nu;
  f.L = gbl(store + s.Loff);
  f.U = gbl(store + s.Uoff);
  f.F = s.nu > 0 ? gbl(scratch + s.Foff) : nullptr;   // Foff may be shifted (block nodes)
  return f;
}

__device__ __forceinline__ gdbl* fel(const FrontPtrs& f, int64_t i, int64_t j) {
  if (j < f.ns) return f.L + j * f.M + i;
  if (i < f.ns) return f.U + (j - f.ns) * f.ns + i;
  return f.F + (j - f.ns) * f.nu + (i - f.ns);
}

// ------------------------------------------------------------------------------------
// Blocked path, step 2: apply the panel's row permutation to every other column of the
// front and compute the U row block  U[kb:kb+w, kb+w:M] = L_kk^{-1} A[kb:kb+w, kb+w:M].
// One workgroup per 64 columns; columns outside the panel are numbered c in [0, M-w):
// col = c < kb ? c : c + w.
// ------------------------------------------------------------------------------------
__device__ __forceinline__ int find_front_tile(const FrontTile* __restrict__ ft, int cnt, int64_t b) {
  int lo = 0, hi = cnt - 1;
  while (lo < hi) {
    int mid = (lo + hi + 1) >> 1;
    if (ft[mid].wg0 <= b) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// Full-width (w == W) triangular solves for one column / row held in registers, with the
// triangle broadcast from LDS.  Each elimination step first issues all of its LDS reads, then
// its FMAs (sched_barrier keeps the scheduler from interleaving them), so the LDS latency is
// paid once per step instead of once per pair of FMAs.  Same operations in the same order as
// the guarded generic loops: results are bitwise identical.
template <int W, int LD = W, int XN = W>
__device__ __forceinline__ void lower_unit_solve_fast(double (&x)[XN], const double* __restrict__ sT) {
  // reads of one step in batches of at most 32 (keeps the kernel within 256 registers so that
  // it can share a SIMD with a resident GEMM wave)
#pragma unroll
  for (int j = 0; j < W - 1; ++j) {
#pragma unroll
    for (int i0 = j + 1; i0 < W; i0 += 32) {
      double lc[32];
#pragma unroll
      for (int i = i0; i < W && i < i0 + 32; ++i) lc[i - i0] = sT[j * LD + i];
      __builtin_amdgcn_sched_barrier(0);
      const double xj = x[j];
#pragma unroll
      for (int i = i0; i < W && i < i0 + 32; ++i) x[i] = fma(-lc[i - i0], xj, x[i]);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
}

// x <- x U^{-1} for a row vector x, U = sT (stored [col][row]), rd = 1/diag(U); returns max |x|
template <int W, int LD = W, int XN = W>
__device__ __forceinline__ double upper_right_solve_fast(double (&x)[XN], const double* __restrict__ sT,
                                                         const double* __restrict__ rd) {
  double gmax = 0.0;
#pragma unroll
  for (int j = 0; j < W; ++j) {
    x[j] = x[j] * rd[j];
    gmax = fmax(gmax, fabs(x[j]));
#pragma unroll
    for (int k0 = j + 1; k0 < W; k0 += 32) {
      double uc[32];
#pragma unroll
      for (int k = k0; k < W && k < k0 + 32; ++k) uc[k - k0] = sT[k * LD + j];
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int k = k0; k < W && k < k0 + 32; ++k) x[k] = fma(-x[j], uc[k - k0], x[k]);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  return gmax;
}

// Two-level blocking: inner panels (nb = 32/64 columns) are grouped in outer blocks of OB = 256
// columns [ostart, oend).  mode 0 (inner step, panel at kb): apply the panel's row swaps to
// every column outside the panel; TRSM only the columns inside the outer block [kb+w, oend).
// mode 1 (outer phase, sub-panel at kb): TRSM rows [kb, kb+w) on the columns right of the
// outer block [oend, M); no swaps (already applied).  kb comes from FrontTile.pad.
__device__ __forceinline__ double readlane_f64(double v, int lane) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), lane);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// LDS hand-off inside one wave (no workgroup barrier): stores complete and become visible to
// the wave's later loads, and the compiler may not move LDS accesses across it.
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// Substitution over one 64x64 diagonal block of a large front for a vector held one element per
// lane (lanes >= bw hold finite values, e.g. 0).  row: this lane's row of the block strictly below
// (forward, unit diagonal) or strictly above (backward) the diagonal, zero elsewhere, loaded into
// registers up front -- so every step is one broadcast and one fma over all lanes (lanes outside
// the triangle add an exact zero) with no exec-mask changes, and the dependent chain per step is
// readlane + fma.  Backward: column j of row pre-scaled by 1/u_jj (tri64_scale_upper), x_i = xi_i /
// u_ii applied once at the end (dinv = this lane's 1/u_ii).  Shared by k_tri_block and k_tri_sweep
// (bitwise equal schedules).
template <bool UPPER, class RJ>
__device__ __forceinline__ double tri64_acc(double xi, RJ&& row, double dinv, int bw) {
  if (bw == 64) {   // full block (all but a front's last): no per-step guard in the chain
    if (!UPPER) {
#pragma unroll
      for (int j = 0; j < 64; ++j) xi = fma(-row(j), readlane_f64(xi, j), xi);
      return xi;
    }
#pragma unroll
    for (int j = 63; j >= 0; --j) xi = fma(-row(j), readlane_f64(xi, j), xi);
    return xi * dinv;
  }
  if (!UPPER) {
#pragma unroll
    for (int j = 0; j < 64; ++j)
      if (j < bw) xi = fma(-row(j), readlane_f64(xi, j), xi);
    return xi;
  }
#pragma unroll
  for (int j = 63; j >= 0; --j)
    if (j < bw) xi = fma(-row(j), readlane_f64(xi, j), xi);
  return xi * dinv;
}
template <bool UPPER>
__device__ __forceinline__ double tri64_row(double xi, const double (&row)[64], double dinv, int bw) {
  return tri64_acc<UPPER>(xi, [&](int j) { return row[j]; }, dinv, bw);
}
// The same substitution for NR right-hand sides at once, the NR chains interleaved step by step
// (independent readlane + fma chains keep the fp64 pipe busy: a batched chain costs about twice a
// single one instead of NR times).  Per right-hand side the operations and their order are
// tri64_row's, so every column is bitwise the single-vector result.
template <bool UPPER, int NR>
__device__ __forceinline__ void tri64_rows(double (&xi)[NR], const double (&row)[64], double dinv, int bw) {
  if (bw == 64) {
#pragma unroll
    for (int jj = 0; jj < 64; ++jj) {
      const int j = UPPER ? 63 - jj : jj;
#pragma unroll
      for (int r = 0; r < NR; ++r) xi[r] = fma(-row[j], readlane_f64(xi[r], j), xi[r]);
    }
  } else {
#pragma unroll
    for (int jj = 0; jj < 64; ++jj) {
      const int j = UPPER ? 63 - jj : jj;
      if (j < bw)
#pragma unroll
        for (int r = 0; r < NR; ++r) xi[r] = fma(-row[j], readlane_f64(xi[r], j), xi[r]);
    }
  }
  if (UPPER)
#pragma unroll
    for (int r = 0; r < NR; ++r) xi[r] *= dinv;
}
// row[j] *= 1/u_jj (held by lane j as dinv), j < bw: the backward row for tri64_row.
__device__ __forceinline__ void tri64_scale_upper(double (&row)[64], double dinv, int bw) {
#pragma unroll
  for (int j = 0; j < 64; ++j)
    if (j < bw) row[j] *= readlane_f64(dinv, j);
}
// This lane's row of the diagonal block D (ld M) for tri64_row: its strictly lower / upper part.
template <bool UPPER>
__device__ __forceinline__ void load_tri_row64(double (&row)[64], const double* __restrict__ D, int64_t M, int bw,
                                               int lane) {
#pragma unroll
  for (int j = 0; j < 64; ++j)
    row[j] = (lane < bw && j < bw && (UPPER ? j > lane : j < lane)) ? D[(int64_t)j * M + lane] : 0.0;
}
__device__ __forceinline__ double diag_recip(const double* __restrict__ D, int64_t M, int bw, int lane) {
  return lane < bw ? recip(D[(int64_t)lane * M + lane]) : 1.0;
}

// sum_{j < bw} d[j] * xj(j) as eight interleaved partial sums (j mod 8) combined pairwise: the
// dependent fp64 chain is 8 + 3 operations deep instead of 64 (~32 cycles each on gfx950).  The
// one row-block product of the large-front solves (k_tri_block, k_tri_sweep), so a column of a
// batched solve stays bitwise equal to the single-vector solve.
template <class XJ>
__device__ __forceinline__ double dot64_split(const double (&d)[64], int bw, XJ&& xj) {
  double a[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) a[k] = 0.0;
#pragma unroll
  for (int j = 0; j < 64; ++j)
    if (j < bw) a[j & 7] = fma(d[j], xj(j), a[j & 7]);
  return ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
}

// acc += sum_{j < bw} D[j*M + i] * xs[j] (bw <= 64) in ascending j: all loads issued up front.
__device__ __forceinline__ double dot64(const double* __restrict__ D, int64_t M, int64_t i, int bw,
                                        const double* __restrict__ xs, double acc) {
  double d[64];
#pragma unroll
  for (int j = 0; j < 64; ++j) d[j] = j < bw ? D[(int64_t)j * M + i] : 0.0;
#pragma unroll
  for (int j = 0; j < 64; ++j)
    if (j < bw) acc = fma(d[j], xs[j], acc);
  return acc;
}

}  // namespace smlu
