// kernels_gemm.hip — dense fp64 Schur-complement updates C -= A*B (MFMA 128 and 64 tiles; the VALU
// 64 tile k_gemm is the bitwise comparison tile and the use_mfma = 0 path).
#include "kernels_common.hpp"

namespace smlu {

// ------------------------------------------------------------------------------------
// Dense update C -= A*B (fp64 VALU).  64x64 output tile per 256-thread workgroup, 4x4 per
// thread, K staged through LDS in slices of 16 with register prefetch of the next slice.
// ------------------------------------------------------------------------------------
__device__ __forceinline__ int find_gemm_task(const GemmTask* __restrict__ t, int cnt, int64_t b) {
  int lo = 0, hi = cnt - 1;
  while (lo < hi) {
    int mid = (lo + hi + 1) >> 1;
    if (t[mid].tile0 <= b) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}


// Tile placement.  (1) XCD-aware remap (bijective for any grid): the workgroups that share an
// XCD (same blockIdx % 8) get one contiguous range of tile indices; with in-order dispatch the
// tiles an XCD runs at the same time are then neighbours.  (2) Grouped order inside a task:
// groups of 8 tile rows, column-major inside a group, so 64 neighbouring tiles form an 8 x 8
// block of C and share 8 A row blocks and 8 B column blocks in that XCD's L2.
__device__ __forceinline__ int64_t xcd_remap(int64_t b, int64_t nwg) {
  const int64_t q = nwg >> 3, r = nwg & 7, x = b & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b >> 3);
}
// Windowed XCD-aware placement for launches whose tasks differ in cost (the batched F22 updates:
// thousands of small-k tasks next to a few large-k ones).  Blocks are dealt round-robin to the 8
// XCDs and roughly 512 run at a time (256 CUs x 2), so within each window of 512 blocks the 64 of
// one XCD take 64 consecutive tiles (one 8 x 8 group of tile_rc: shared A and B panels in that L2),
// while consecutive groups go to different XCDs: every XCD gets a share of every task.  (xcd_remap's
// one contiguous range per XCD left XCDs idle behind the large-k tasks.)  Bijective; a partial last
// window keeps dispatch order.
__device__ __forceinline__ int64_t xcd_window_remap(int64_t b, int64_t nwg) {
  constexpr int64_t W = 512;
  if (b >= (nwg / W) * W) return b;
  const int64_t w0 = b - b % W, i = b % W;
  return w0 + (i & 7) * (W / 8) + (i >> 3);
}
template <int TS>
__device__ __forceinline__ void tile_rc(const GemmTask& t, int64_t tl, int& tm, int& tn) {
  constexpr int GM = 8;
  const int64_t tiles_n = (t.n + TS - 1) / TS;
  const int64_t g = tl / (GM * tiles_n);
  const int first = (int)(g * GM);
  const int gm = min(GM, t.tiles_m - first);
  const int64_t in = tl - g * GM * tiles_n;
  tm = first + (int)(in % gm);
  tn = (int)(in / gm);
}

// Growth check of a GEMM-form triangular solve (task.gsid >= 0): max |result| of the tile, folded
// into growth[0] and the front's weak-pivot bit exactly as k_step_trsm does for its L rows.
struct GrowthArgs {
  int32_t* info;
  double* growth;
  double piv_tol;
};
__device__ __forceinline__ void tile_growth(const GrowthArgs& ga, int sid, double g) {
  g = wave_max(g);
  if ((threadIdx.x & 63) == 0 && g > 0.0) {
    atomic_max_pos(&ga.growth[0], g);
    if (g > 1.0 / ga.piv_tol) atomicOr(&ga.info[sid], 2);
  }
}

#define GBM 64
#define GBN 64
#define GBK 16
// TRSM = true: the GEMM-form triangular-solve launches (growth epilogue; a separate symbol so
// that profiles tell them apart from the Schur-complement updates)
template <bool TRSM>
__global__ __launch_bounds__(256) void k_gemm(const GemmTask* __restrict__ tasks, int ntask, GrowthArgs ga) {
  __shared__ double As[2][GBK][GBM + 2];
  __shared__ double Bs[2][GBK][GBN + 2];
  const int64_t b = xcd_remap(blockIdx.x, gridDim.x);
  const GemmTask t = tasks[find_gemm_task(tasks, ntask, b)];
  const gdbl* gA = gbl(t.A);
  const gdbl* gB = gbl(t.B);
  gdbl* gC = gbl(t.C);
  int tm, tn;
  tile_rc<GBM>(t, b - t.tile0, tm, tn);
  const int m0 = tm * GBM, n0 = tn * GBN;
  const int tid = threadIdx.x;
  const int tx = tid & 15, ty = tid >> 4;  // 16 x 16 threads, 4x4 each
  // accumulators start from C (its loads overlap the first K slice's), B is staged negated:
  // acc = C + sum(A * -B), and the epilogue is stores only
  double acc[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = n0 + ty + 16 * j;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = m0 + tx + 16 * i;
      acc[i][j] = (col < t.n && row < t.m) ? gC[(int64_t)col * t.ldc + row] : 0.0;
    }
  }
  // load mapping: A slice GBM x GBK: thread -> (row = tid & 63, kk = (tid >> 6) + 4*r), r<4
  //               B slice GBK x GBN: thread -> (kk = tid & 15, col = (tid >> 4) + 16*r), r<4
  const int ar = tid & 63, ak = tid >> 6;
  const int bk = tid & 15, bc = tid >> 4;
  double ra[4], rb[4];
  const int K = t.k;
  auto gload = [&](int k0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      int kk = ak + 4 * r;
      int row = m0 + ar;
      ra[r] = (row < t.m && k0 + kk < K) ? gA[(int64_t)(k0 + kk) * t.lda + row] : 0.0;
      int col = n0 + bc + 16 * r;
      rb[r] = (col < t.n && k0 + bk < K) ? gB[(int64_t)col * t.ldb + k0 + bk] : 0.0;
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      As[buf][ak + 4 * r][ar] = ra[r];
      Bs[buf][bk][bc + 16 * r] = -rb[r];
    }
  };
  int nk = (K + GBK - 1) / GBK;
  gload(0);
  sstore(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) gload((kt + 1) * GBK);
#pragma unroll 4
    for (int kk = 0; kk < GBK; ++kk) {
      double a[4], bb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = As[cur][kk][tx + 16 * i];
#pragma unroll
      for (int j = 0; j < 4; ++j) bb[j] = Bs[cur][kk][ty + 16 * j];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = fma(a[i], bb[j], acc[i][j]);
    }
    if (kt + 1 < nk) sstore(cur ^ 1);
    __syncthreads();
  }
  double gmax = 0.0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = n0 + ty + 16 * j;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = m0 + tx + 16 * i;
      if (col < t.n && row < t.m) {
        gC[(int64_t)col * t.ldc + row] = acc[i][j];
        gmax = fmax(gmax, fabs(acc[i][j]));
      }
    }
  }
  if (TRSM && t.gsid >= 0) tile_growth(ga, t.gsid, gmax);
}

// The same 64 x 64 tile on the fp64 matrix cores (tile code 66, the default for k > 64 launches
// below the 128-tile threshold; SMLU_SMALLK=0 keeps k_gemm): identical staging and slices, each
// wave a 32 x 32 quadrant of 2 x 2 v_mfma_f64_16x16x4 blocks (lane l of block (i, j) holds
// C[16 i + (l & 15)][16 j + (l >> 4) + 4 r]); per element one fused multiply-add per k in
// ascending order, bitwise k_gemm's result.
typedef double v4d __attribute__((ext_vector_type(4)));
template <bool TRSM>
__global__ __launch_bounds__(256) void k_gemm64_mfma(const GemmTask* __restrict__ tasks, int ntask, GrowthArgs ga) {
  __shared__ double As[2][GBK][GBM + 2];
  __shared__ double Bs[2][GBK][GBN + 2];
  const int64_t b = xcd_remap(blockIdx.x, gridDim.x);
  const GemmTask t = tasks[find_gemm_task(tasks, ntask, b)];
  const gdbl* gA = gbl(t.A);
  const gdbl* gB = gbl(t.B);
  gdbl* gC = gbl(t.C);
  int tm, tn;
  tile_rc<GBM>(t, b - t.tile0, tm, tn);
  const int m0 = tm * GBM, n0 = tn * GBN;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = (wv & 1) * 32, wc = (wv >> 1) * 32;
  const int li = lane & 15, lk = lane >> 4;
  v4d acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = m0 + wr + 16 * i + li;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int col = n0 + wc + 16 * j + lk + 4 * r;
        acc[i][j][r] = (col < t.n && row < t.m) ? gC[(int64_t)col * t.ldc + row] : 0.0;
      }
  }
  const int ar = tid & 63, ak = tid >> 6;
  const int bk = tid & 15, bc = tid >> 4;
  double ra[4], rb[4];
  const int K = t.k;
  auto gload = [&](int k0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int kk = ak + 4 * r;
      const int row = m0 + ar;
      ra[r] = (row < t.m && k0 + kk < K) ? gA[(int64_t)(k0 + kk) * t.lda + row] : 0.0;
      const int col = n0 + bc + 16 * r;
      rb[r] = (col < t.n && k0 + bk < K) ? gB[(int64_t)col * t.ldb + k0 + bk] : 0.0;
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      As[buf][ak + 4 * r][ar] = ra[r];
      Bs[buf][bk][bc + 16 * r] = -rb[r];
    }
  };
  const int nk = (K + GBK - 1) / GBK;
  gload(0);
  sstore(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) gload((kt + 1) * GBK);
#pragma unroll
    for (int kq = 0; kq < GBK / 4; ++kq) {
      const int k = 4 * kq + lk;
      double fa[2], fb[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) fa[i] = As[cur][k][wr + 16 * i + li];
#pragma unroll
      for (int j = 0; j < 2; ++j) fb[j] = Bs[cur][k][wc + 16 * j + li];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(fb[j], fa[i], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) sstore(cur ^ 1);
    __syncthreads();
  }
  double gmax = 0.0;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = m0 + wr + 16 * i + li;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int col = n0 + wc + 16 * j + lk + 4 * r;
        if (col < t.n && row < t.m) {
          gC[(int64_t)col * t.ldc + row] = acc[i][j][r];
          gmax = fmax(gmax, fabs(acc[i][j][r]));
        }
      }
  }
  if (TRSM && t.gsid >= 0) tile_growth(ga, t.gsid, gmax);
}

// Small-k variant of k_gemm (every task of the launch has k <= 64: the in-block updates and the
// GEMM-form triangular solves): the whole K extent of the A and B tiles is staged in one shot
// (32 loads per thread in flight together with the 16 C loads), so a launch pays one memory
// round trip instead of one per 16-deep slice.  Same per-element arithmetic as k_gemm.
// One 64 x 64 output tile [m0, m0+64) x [n0, n0+64) of an m x n task (k <= 64), by the whole
// 256-thread workgroup; returns the thread's max |result| (growth epilogue of the TRSM form).
// All loads (C, A, B) complete before the first store, so B == C (in place) is allowed.
// On the fp64 matrix cores (round 5; the VALU form it replaced took 1.1 ms more in-block update
// and 1.6 ms more GEMM-form TRSM time per 128^3 refactor): each wave a 32 x 32 quadrant of 2 x 2
// v_mfma_f64_16x16x4 blocks over the staged A / -B images (lane l of block (i, j) holds
// C[16 i + (l & 15)][16 j + (l >> 4) + 4 r]).  Per element the MFMA's chain is one fused
// multiply-add per k in ascending order, the zero-filled k >= K terms exact no-ops: bitwise the
// VALU tiles' result.
__device__ __forceinline__ double k64_tile_mfma(const gdbl* gA, int lda, const gdbl* gB, int ldb, gdbl* gC, int ldc,
                                                int m, int n, int K, int m0, int n0,
                                                double (&As)[64][GBM + 2], double (&Bs)[64][GBN + 2]) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = (wv & 1) * 32, wc = (wv >> 1) * 32;
  const int li = lane & 15, lk = lane >> 4;
  v4d acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = m0 + wr + 16 * i + li;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int col = n0 + wc + 16 * j + lk + 4 * r;
        acc[i][j][r] = (col < n && row < m) ? gC[(int64_t)col * ldc + row] : 0.0;
      }
  }
  // A: row = tid & 63, k = (tid >> 6) + 4r;  B: k = tid & 63, col = (tid >> 6) + 4r
  const int ar = tid & 63, ak = tid >> 6;
  double ra[16], rb[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int kk = ak + 4 * r, row = m0 + ar;
    ra[r] = (row < m && kk < K) ? gA[(int64_t)kk * lda + row] : 0.0;
    const int col = n0 + ak + 4 * r;
    rb[r] = (col < n && ar < K) ? gB[(int64_t)col * ldb + ar] : 0.0;
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    As[ak + 4 * r][ar] = ra[r];
    Bs[ar][ak + 4 * r] = -rb[r];
  }
  __syncthreads();
  auto kquad = [&](int kq) {
    const int k = 4 * kq + lk;
    double fa[2], fb[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) fa[i] = As[k][wr + 16 * i + li];
#pragma unroll
    for (int j = 0; j < 2; ++j) fb[j] = Bs[k][wc + 16 * j + li];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(fb[j], fa[i], acc[i][j], 0, 0, 0);
  };
  if (K == 64) {   // full panels (w = 64): straight-line
#pragma unroll
    for (int kq = 0; kq < 16; ++kq) kquad(kq);
  } else {
    const int nkq = (K + 3) >> 2;
    for (int kq = 0; kq < nkq; ++kq) kquad(kq);
  }
  double gmax = 0.0;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = m0 + wr + 16 * i + li;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int col = n0 + wc + 16 * j + lk + 4 * r;
        if (col < n && row < m) {
          gC[(int64_t)col * ldc + row] = acc[i][j][r];
          gmax = fmax(gmax, fabs(acc[i][j][r]));
        }
      }
  }
  return gmax;
}

template <bool TRSM>
__global__ __launch_bounds__(256) void k_gemm_k64(const GemmTask* __restrict__ tasks, int ntask, GrowthArgs ga) {
  __shared__ double As[64][GBM + 2];   // [k][row]
  __shared__ double Bs[64][GBN + 2];   // [k][col], negated
  const int64_t b = xcd_remap(blockIdx.x, gridDim.x);
  const GemmTask t = tasks[find_gemm_task(tasks, ntask, b)];
  int tm, tn;
  tile_rc<GBM>(t, b - t.tile0, tm, tn);
  const double gmax = k64_tile_mfma(gbl(t.A), t.lda, gbl(t.B), t.ldb, gbl(t.C), t.ldc, t.m, t.n, t.k, tm * GBM,
                                    tn * GBN, As, Bs);
  if (TRSM && t.gsid >= 0) tile_growth(ga, t.gsid, gmax);
}

// ------------------------------------------------------------------------------------
// 128 x 128 output tiles on the fp64 matrix cores (opts.use_mfma = 1, the default; use_mfma = 0
// runs every launch on the VALU 64 tile k_gemm), K staged through double-buffered LDS slices of
// 16.  v_mfma_f64_16x16x4_f64; each wave owns a 64x64 quadrant = 4x4
// blocks.  The product is formed as C^T = B^T A^T so that the accumulator's lane index runs
// along C's rows (column-major C stays coalesced): lane l of block (bi,bj) holds
// C[row = 16 bi + (l & 15)][col = 16 bj + (l >> 4) + 4 r], r = 0..3.
#define HBM_ 128
#define HBK_ 16
#define HLDB_ (HBM_ + 2)
// Guard-free operand and C traffic on interior tiles (m, n in range), K guards only in the
// last, partial slice (FULL = false: every access guarded).  +1-4 % over the guarded form
// (k = 384 trailing shapes 48.4 -> 50.1 TFLOP/s, tools/gemm_bench).
template <bool TRSM, bool FULL>
__device__ __forceinline__ void gemm128_mfma_body(const GemmTask& t, int m0, int n0,
                                                double (&As)[2][HBK_][HBM_], double (&Bs)[2][HBK_][HLDB_],
                                                const GrowthArgs& ga) {
  const gdbl* gA = gbl(t.A);
  const gdbl* gB = gbl(t.B);
  gdbl* gC = gbl(t.C);
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wr = (wv & 1) * 64, wc = (wv >> 1) * 64;
  const int li = lane & 15, lk = lane >> 4;
  v4d acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = m0 + wr + 16 * i + li;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int col = n0 + wc + 16 * j + lk + 4 * r;
        acc[i][j][r] = (FULL || (row < t.m && col < t.n)) ? gC[(int64_t)col * t.ldc + row] : 0.0;
      }
  }
  const int ar = tid & 127, ak = tid >> 7;
  const int bk = tid & 15, bc = tid >> 4;
  const int K = t.k;
  const int arow = m0 + ar;
  const bool arow_ok = FULL || arow < t.m;
  const gdbl* Ap = gA + arow;
  const gdbl* Bp = gB + (int64_t)(n0 + bc) * t.ldb + bk;
  double ra[8], rb[8];
  auto gload = [&](int k0, bool kguard) {
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int kk = k0 + ak + 2 * r;
      if (!kguard && FULL) ra[r] = Ap[(int64_t)kk * t.lda];
      else ra[r] = (arow_ok && kk < K) ? Ap[(int64_t)kk * t.lda] : 0.0;
      const int col = n0 + bc + 16 * r;
      if (!kguard && FULL) rb[r] = Bp[(int64_t)16 * r * t.ldb + k0];
      else rb[r] = ((FULL || col < t.n) && k0 + bk < K) ? Bp[(int64_t)16 * r * t.ldb + k0] : 0.0;
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      As[buf][ak + 2 * r][ar] = ra[r];
      Bs[buf][bk][bc + 16 * r] = -rb[r];
    }
  };
  const int nk = (K + HBK_ - 1) / HBK_;
  const int nfull = K / HBK_;   // slices with every k in range
  gload(0, nfull == 0);
  sstore(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) gload((kt + 1) * HBK_, kt + 1 >= nfull);
#pragma unroll
    for (int kq = 0; kq < HBK_ / 4; ++kq) {
      const int k = kq * 4 + lk;
      double fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = As[cur][k][wr + 16 * i + li];
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = Bs[cur][k][wc + 16 * j + li];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(fb[j], fa[i], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) sstore(cur ^ 1);
    __syncthreads();
  }
  double gmax = 0.0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = m0 + wr + 16 * i + li;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int col = n0 + wc + 16 * j + lk + 4 * r;
        if (FULL || (row < t.m && col < t.n)) {
          gC[(int64_t)col * t.ldc + row] = acc[i][j][r];
          if (TRSM) gmax = fmax(gmax, fabs(acc[i][j][r]));
        }
      }
  }
  if (TRSM && t.gsid >= 0) tile_growth(ga, t.gsid, gmax);
}


// Pair types and global accessors of the v3 tile.
typedef double v2du __attribute__((ext_vector_type(2), aligned(8)));   // 8-byte aligned pairs (global)
typedef double v2d __attribute__((ext_vector_type(2)));                 // 16-byte aligned pairs (LDS)
// Global accesses: wave-uniform 64-bit base (SGPRs, recomputed by scalar ALU where used) + a
// per-lane 32-bit byte offset fixed for the whole tile, so no 64-bit per-lane address is live
// across the K loop (the v1 interior spilled its precomputed C addresses).
__device__ __forceinline__ v2d ldu2(const char* ubase, uint32_t off) {
  return *(const __attribute__((address_space(1))) v2du*)(ubase + off);
}
__device__ __forceinline__ void stu2(char* ubase, uint32_t off, v2d v) {
  *(__attribute__((address_space(1))) v2du*)(ubase + off) = v;
}

// ------------------------------------------------------------------------------------
// MFMA tile v3 (tile code 131): the v2 tile's output mapping and per-element arithmetic (acc = C,
// then one fp64 MFMA-FMA per k in ascending k: bitwise identical to v2 and the VALU tiles), with
// the K slices staged by LDS-DMA instead of registers:
//  * global_load_lds_dwordx4 (16 bytes per lane, lane-linear LDS destination): A as k-rows of
//    128 doubles (one 1 KB row per wave instruction, the v2 image [k][row]); B as 8 columns x 16 k
//    per wave instruction, image [col][k] with the k pairs of column c stored at pair slot
//    p ^ ((c >> 1) & 7) (the swizzle is applied to the per-lane SOURCE address, the LDS side stays
//    lane-linear), which makes the fragment reads -- 16 consecutive columns at one k per
//    half-wave -- bank-conflict free;
//  * B's sign flip is the MFMA's own neg modifier on the B fragment (exact: -b*a = b*(-a)), so no
//    staging VALU work and no staging registers: the 32 VGPRs v2 spent on the in-flight slice
//    hold a second fragment set instead, and the fragments of k-quad q+1 are read while the 16
//    MFMAs of quad q run;
//  * one barrier per slice, which also retires the slice's DMA (the next slice's DMA is issued
//    at the top of the current slice, into the other buffer, whose readers passed the previous
//    barrier);
//  * a partial last slice (K % 16) is staged through registers with zero fill, into the same
//    images (no guard in the compute loop).
// Interior tiles only; edge tiles take gemm128_mfma_body<.., false> (same arithmetic).
// ------------------------------------------------------------------------------------
struct Mfma3Lds {
  double A[2][HBK_][HBM_];   // [buf][k][row]
  double B[2][HBM_][HBK_];   // [buf][col][k, pair-swizzled]
};
static_assert(sizeof(Mfma3Lds) == 65536, "v3 tile LDS image");
typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ void glds16(const void* src, void* lds_dst) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src, (lds_void*)lds_dst, 16, 0, 0);
}


template <bool TRSM, bool EB>
__device__ __forceinline__ void gemm128_mfma3_interior(const GemmTask& t, int m0, int n0, Mfma3Lds& S,
                                                       const GrowthArgs& ga) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = (wv & 1) * 64, wc = (wv >> 1) * 64;
  const int li = lane & 15, lk = lane >> 4;
  const int K = t.k;
  const int64_t lda = t.lda, ldb = t.ldb, ldc = t.ldc;
  const uint32_t c_lo = (uint32_t)(((int64_t)lk * ldc + 2 * li) * 8);
  auto cbase = [&](int ip, int j, int r) {
    return reinterpret_cast<char*>(t.C) + ((int64_t)(n0 + wc + 16 * j + 4 * r) * ldc + m0 + wr + 32 * ip) * 8;
  };
  // DMA sources of this lane.  A: k-row wv + 4q of the slice, rows m0 + 2 lane, +1.
  // B: wave instruction q covers columns 8 (wv + 4q) + [0, 8); lane -> column 8 (wv + 4q) + (lane >> 3),
  //    pair slot lane & 7 holding k pair (lane & 7) ^ ((column >> 1) & 7) = (lane & 7) ^ ((4 wv + (lane >> 4)) & 7).
  const int bpair = (lane & 7) ^ ((4 * wv + (lane >> 4)) & 7);
  const char* asrc = reinterpret_cast<const char*>(t.A) + ((int64_t)wv * lda + m0 + 2 * lane) * 8;
  const char* bsrc = reinterpret_cast<const char*>(t.B) + ((int64_t)(n0 + 8 * wv + (lane >> 3)) * ldb + 2 * bpair) * 8;
  auto issue = [&](int k0, int buf) {   // one full slice (k0 + 16 <= K): 4 + 4 DMA per wave
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      glds16(asrc + ((int64_t)(k0 + 4 * q) * lda) * 8, &S.A[buf][wv + 4 * q][0]);
      glds16(bsrc + ((int64_t)32 * q * ldb + k0) * 8, &S.B[buf][8 * (wv + 4 * q)][0]);
    }
  };
  auto stage_tail = [&](int k0, int buf) {   // partial slice: guarded register loads, zero fill
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int ka = k0 + wv + 4 * q;
      const v2d a = ka < K ? ldu2(asrc + ((int64_t)(k0 + 4 * q) * lda) * 8, 0) : v2d{0.0, 0.0};
      *reinterpret_cast<v2d*>(&S.A[buf][wv + 4 * q][2 * lane]) = a;
      const gdbl* bp = gbl(reinterpret_cast<const double*>(bsrc + ((int64_t)32 * q * ldb + k0) * 8));
      const int kb = k0 + 2 * bpair;
      v2d b;
      b.x = kb < K ? bp[0] : 0.0;
      b.y = kb + 1 < K ? bp[1] : 0.0;
      *reinterpret_cast<v2d*>(&S.B[buf][8 * (wv + 4 * q)][2 * lane]) = b;
    }
  };
  v4d acc[4][4];
#pragma unroll
  for (int ip = 0; ip < 2; ++ip)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const v2d c = ldu2(cbase(ip, j, r), c_lo);
        acc[2 * ip][j][r] = c.x;
        acc[2 * ip + 1][j][r] = c.y;
      }
  // fragment addresses: A row pair wr + 32 ip + 2 li at k = 4 kq + lk; B column wc + 16 j + li at
  // k = 4 kq + lk, i.e. pair 2 kq + (lk >> 1), slot that ^ (li >> 1), element lk & 1
  const int a_off = (lk * HBM_ + wr + 2 * li);
  int b_off[4];
#pragma unroll
  for (int kq = 0; kq < 4; ++kq) b_off[kq] = (wc + li) * HBK_ + (((2 * kq + (lk >> 1)) ^ (li >> 1)) << 1) + (lk & 1);
  auto frags = [&](int cur, int kq, v2d (&fa)[2], double (&fb)[4]) {
    const double* As = &S.A[cur][0][0] + a_off + kq * 4 * HBM_;
    const double* Bs = &S.B[cur][0][0] + b_off[kq];
#pragma unroll
    for (int ip = 0; ip < 2; ++ip) fa[ip] = *reinterpret_cast<const v2d*>(As + 32 * ip);
#pragma unroll
    for (int j = 0; j < 4; ++j) fb[j] = Bs[16 * HBK_ * j];
  };
  auto quad = [&](const v2d (&fa)[2], const double (&fb)[4]) {
#pragma unroll
    for (int ip = 0; ip < 2; ++ip)
#pragma unroll
      for (int j = 0; j < 4; ++j) {   // neg:[1,0,0]: C - B*A
        acc[2 * ip][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(fb[j], fa[ip].x, acc[2 * ip][j], 0, 0, 1);
        acc[2 * ip + 1][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(fb[j], fa[ip].y, acc[2 * ip + 1][j], 0, 0, 1);
      }
  };
  auto slice = [&](int cur) {
    v2d fa0[2], fa1[2];
    double fb0[4], fb1[4];
    frags(cur, 0, fa0, fb0);
    frags(cur, 1, fa1, fb1);
    quad(fa0, fb0);
    frags(cur, 2, fa0, fb0);
    quad(fa1, fb1);
    frags(cur, 3, fa1, fb1);
    quad(fa0, fb0);
    quad(fa1, fb1);
  };
  const int nk = (K + HBK_ - 1) / HBK_;
  const int nfull = K / HBK_;
  if (nfull > 0) issue(0, 0);
  else stage_tail(0, 0);
  __syncthreads();
  if (!EB) {
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      const bool next = kt + 1 < nk;
      const bool next_full = kt + 1 < nfull;
      if (next_full) issue((kt + 1) * HBK_, cur ^ 1);
      if (next && !next_full) stage_tail((kt + 1) * HBK_, cur ^ 1);
      slice(cur);
      if (next) __syncthreads();
    }
  } else {
    // the next slice's barrier between k-quads 2 and 3 (all of this slice's fragments are in
    // registers by then) and its first fragments read behind quad 3's MFMAs
    v2d fa0[2], fa1[2];
    double fb0[4], fb1[4];
    frags(0, 0, fa0, fb0);
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      const bool next = kt + 1 < nk;
      const bool next_full = kt + 1 < nfull;
      if (next_full) issue((kt + 1) * HBK_, cur ^ 1);
      if (next && !next_full) stage_tail((kt + 1) * HBK_, cur ^ 1);
      frags(cur, 1, fa1, fb1);
      quad(fa0, fb0);
      frags(cur, 2, fa0, fb0);
      quad(fa1, fb1);
      frags(cur, 3, fa1, fb1);
      quad(fa0, fb0);
      if (next) {
        __syncthreads();
        frags(cur ^ 1, 0, fa0, fb0);
      }
      quad(fa1, fb1);
    }
  }
  double gmax = 0.0;
#pragma unroll
  for (int ip = 0; ip < 2; ++ip)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const v2d c = v2d{acc[2 * ip][j][r], acc[2 * ip + 1][j][r]};
        stu2(cbase(ip, j, r), c_lo, c);
        if (TRSM) gmax = fmax(gmax, fmax(fabs(c.x), fabs(c.y)));
      }
  if (TRSM && t.gsid >= 0) tile_growth(ga, t.gsid, gmax);
}

#ifdef SMLU_CLOCK_PROBE
// Dev build only (tools/gemm_clock.py): the shader clock the 128 tile runs at, from the
// workgroup's own counters -- sum of delta s_memtime (shader cycles) and of delta s_memrealtime
// (100 MHz constant clock) over every workgroup of the armed launches, per form (EB = F22, else
// trailing/in-block), accumulated by vector atomics from lane 0.
__device__ unsigned long long* g_clock_probe = nullptr;
struct ClockMark {
  unsigned long long t0, r0;
  __device__ __forceinline__ ClockMark() : t0(__builtin_amdgcn_s_memtime()), r0(__builtin_amdgcn_s_memrealtime()) {}
  __device__ __forceinline__ void done(int form) const {
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    unsigned long long* p = g_clock_probe;
    if (p && threadIdx.x == 0) {
      atomicAdd(p + 4 * form, t1 - t0);
      atomicAdd(p + 4 * form + 1, r1 - r0);
      atomicAdd(p + 4 * form + 2, 1ull);
    }
  }
};
#endif
template <bool TRSM, bool EB = false>
__global__ __launch_bounds__(256, 2) void k_gemm128_mfma3(const GemmTask* __restrict__ tasks, int ntask,
                                                          GrowthArgs ga) {
#ifdef SMLU_CLOCK_PROBE
  const ClockMark mark;
#endif
  __shared__ __attribute__((aligned(16))) double lds[sizeof(Mfma3Lds) / sizeof(double)];
  const int64_t b = xcd_window_remap(blockIdx.x, gridDim.x);
  const GemmTask t = tasks[find_gemm_task(tasks, ntask, b)];
  int tm, tn;
  tile_rc<HBM_>(t, b - t.tile0, tm, tn);
  const int m0 = tm * HBM_, n0 = tn * HBM_;
  if (m0 + HBM_ <= t.m && n0 + HBM_ <= t.n) {
    gemm128_mfma3_interior<TRSM, EB>(t, m0, n0, *reinterpret_cast<Mfma3Lds*>(lds), ga);
  } else {
    auto& As = *reinterpret_cast<double(*)[2][HBK_][HBM_]>(lds);
    auto& Bs = *reinterpret_cast<double(*)[2][HBK_][HLDB_]>(lds + 2 * HBK_ * HBM_);
    gemm128_mfma_body<TRSM, false>(t, m0, n0, As, Bs, ga);
  }
#ifdef SMLU_CLOCK_PROBE
  mark.done(EB ? 0 : 1);
#endif
}

// ------------------------------------------------------------------------------------
// U rows of an outer block, fused (the end-of-block step of the GEMM-form fronts).  One
// 256-thread workgroup per 32-column block of the columns right of the block (L-panel columns or
// U12 columns) runs the whole sub-panel sequence on its columns with the block REGISTER-RESIDENT:
// the OB rows [ob0, ob1) x 32 columns (up to 384 x 32) are loaded once -- wave wv holds the 16-row
// blocks wv, wv + 4, ..., so sub-panel u's four row blocks are one per wave -- and for each 64-row
// sub-panel u:
//   T: C_u <- C_u - NL_u C_u (NL_u = I - L_uu^-1, tinv slot0 + u): the owner waves publish -C_u
//      in LDS, apply the MFMA GEMM form in their registers, publish the new -C_u;
//   R: every wave updates its row blocks below u inside the block, C_r -= L_ru C_u (k = 64), L
//      fragments straight from HBM/L2 (the next block's in flight during the current one's MFMAs).
// The block is stored once at the end: one HBM round trip per column block instead of one per
// sub-panel (round 4 re-loaded and re-stored the rows below u for every u, a latency chain of
// ~115 us per workgroup).  Per element the same operations in the same order as the per-sub-panel
// launches it replaces (acc = C, then one fp64 MFMA-FMA per k ascending with -C_u as the first
// operand), so the factors are bitwise unchanged.
// ------------------------------------------------------------------------------------
#define UR_NC 32    // columns per workgroup
#define UR_RB 6     // 16-row blocks per wave (OB <= 384 = 4 waves x 6 x 16)
#define UR_LD 36    // LDS row stride of -C_u [k][col] (doubles)
// c ? x : +0.0 as a bit mask (keeps the compiler from sinking the load into a branch)
__device__ __forceinline__ double sel0(bool c, double x) {
  return __longlong_as_double(__double_as_longlong(x) & (c ? -1LL : 0LL));
}
__global__ __launch_bounds__(256, 2) void k_urows(const URowTask* __restrict__ tasks, const SNode* __restrict__ sn,
                                                  double* __restrict__ store, const double* __restrict__ tinv) {
  __shared__ double Bs[64 * UR_LD];
  const URowTask t = tasks[blockIdx.x];
  const SNode s = sn[t.s];
  const int64_t M = (int64_t)s.ns + s.nu;
  const int64_t ld = t.ld;
  const int nc = t.ncols;                 // <= 32
  const int nrows = t.ob1 - t.ob0;        // <= 384
  const int tid = threadIdx.x, lane = tid & 63, li = lane & 15, lk = lane >> 4;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  gdbl* const C = gbl(store + t.coff);   // (row, col) at col * ld + row
  const gdbl* const Lp = gbl(store + s.Loff);
  // this lane's element r of block (i, cb): row ob0 + 16 (wv + 4 i) + li, column 16 cb + lk + 4 r
  v4d acc[UR_RB][2];
#pragma unroll
  for (int i = 0; i < UR_RB; ++i) {
    const int lr = 16 * (wv + 4 * i) + li;
    const bool rin = lr < nrows;
    const int row = t.ob0 + (rin ? lr : 0);
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int col = 16 * cb + lk + 4 * r;
        const bool in = rin && col < nc;
        acc[i][cb][r] = sel0(in, C[(int64_t)(in ? col : 0) * ld + row]);
      }
  }
  // -C_u of this wave's block i into the LDS image [k = row within the sub-panel][col]
  auto publish = [&](int i) {
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int r = 0; r < 4; ++r) Bs[(16 * wv + li) * UR_LD + 16 * cb + lk + 4 * r] = -acc[i][cb][r];
  };
  const int nsub = (nrows + 63) >> 6;
#pragma unroll 1
  for (int u = 0; u < nsub; ++u) {
    const int kbu = t.ob0 + 64 * u;
    const int wu = min(64, t.ob1 - kbu);
    const int nkq = (wu + 3) >> 2;
    // ---- T: the four row blocks of sub-panel u are block i = u of each wave
    v4d tc[2];
#pragma unroll
    for (int i = 0; i < UR_RB; ++i)
      if (i == u) {
        publish(i);
        tc[0] = acc[i][0];
        tc[1] = acc[i][1];
      }
    // the wave's NL fragments (rows 16 wv + li of NL_u), all 16 k-quads in flight
    double na[16];
    {
      const gdbl* pn = gbl(tinv + (int64_t)(t.slot0 + u) * 8192) + lk * 64 + 16 * wv + li;
#pragma unroll
      for (int kq = 0; kq < 16; ++kq) na[kq] = sel0(16 * wv + li < wu && 4 * kq + lk < wu, pn[256 * kq]);
    }
    __syncthreads();   // -C_u published
#pragma unroll
    for (int kq = 0; kq < 16; ++kq) {
      if (kq >= nkq) continue;
      const int k = 4 * kq + lk;
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
        tc[cb] = __builtin_amdgcn_mfma_f64_16x16x4f64(Bs[k * UR_LD + 16 * cb + li], na[kq], tc[cb], 0, 0, 0);
    }
    __syncthreads();   // every wave is done reading the old -C_u
#pragma unroll
    for (int i = 0; i < UR_RB; ++i)
      if (i == u) {
        acc[i][0] = tc[0];
        acc[i][1] = tc[1];
        publish(i);
      }
    __syncthreads();   // new -C_u published
    // ---- R: this wave's row blocks below sub-panel u (blocks i > u), C_r -= L_ru C_u
    double fa[16], fn[16];
    auto lfrag = [&](int i, double (&f)[16]) {
      const int lr = 16 * (wv + 4 * i) + li;
      const bool rin = lr < nrows;
      const gdbl* pa = Lp + (int64_t)(kbu + lk) * M + t.ob0 + (rin ? lr : 0);
#pragma unroll
      for (int kq = 0; kq < 16; ++kq) {
        const bool kin = 4 * kq + lk < wu;
        f[kq] = sel0(rin && kin, pa[kin ? (int64_t)4 * kq * M : 0]);
      }
    };
    if (u + 1 < UR_RB && 16 * (wv + 4 * (u + 1)) < nrows) lfrag(u + 1, fa);
#pragma unroll
    for (int i = 1; i < UR_RB; ++i) {
      if (i <= u || 16 * (wv + 4 * i) >= nrows) continue;
      const bool more = i + 1 < UR_RB && 16 * (wv + 4 * (i + 1)) < nrows;
      if (more) lfrag(i + 1, fn);
#pragma unroll
      for (int kq = 0; kq < 16; ++kq) {
        if (kq >= nkq) continue;
        const int k = 4 * kq + lk;
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
          acc[i][cb] = __builtin_amdgcn_mfma_f64_16x16x4f64(Bs[k * UR_LD + 16 * cb + li], fa[kq], acc[i][cb], 0, 0, 0);
      }
      if (more)
#pragma unroll
        for (int kq = 0; kq < 16; ++kq) fa[kq] = fn[kq];
    }
    __syncthreads();   // Bs free for the next sub-panel
  }
#pragma unroll
  for (int i = 0; i < UR_RB; ++i) {
    const int lr = 16 * (wv + 4 * i) + li;
    if (16 * (wv + 4 * i) >= nrows) continue;
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int col = 16 * cb + lk + 4 * r;
        if (lr < nrows && col < nc) C[(int64_t)col * ld + t.ob0 + lr] = acc[i][cb][r];
      }
  }
}

// ------------------------------------------------------------------------------------
// Inverses of a factored 64 x 64 diagonal tile for the GEMM-form triangular solves:
//   NL = I - L_kk^{-1} (L unit lower: the strictly lower part of the tile),
//   NU = I - U_kk^{-1} (U upper with its diagonal),
// column-major with ld 64 at tinv + slot * 8192 (NL) and + 4096 (NU).  A partial panel
// (w < 64) is padded with the identity, so NL/NU vanish outside the w x w block.
// 8 workgroups per front (4 for NL, 4 for NU); a wave computes 4 columns at once by column
// sweep: lane i holds row i, step j broadcasts the finished entry j by v_readlane and every
// lane below (L) / above (U) subtracts its tile entry times it -- one LDS read feeds 4 FMAs.
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_tri_inv(const int32_t* __restrict__ list, int step,
                                                 const SNode* __restrict__ sn,
                                                 double* __restrict__ store,
                                                 double* __restrict__ scratch,
                                                 double* __restrict__ tinv) {
  __shared__ double sD[64 * 65];   // tile [col][row], ld 65
  const int item = blockIdx.x >> 3, part = blockIdx.x & 7;
  const int sid = list[2 * item];
  const int64_t slot = list[2 * item + 1];
  const SNode s = sn[sid];
  FrontPtrs f = front_ptrs(s, store, scratch);
  const int64_t M = f.M;
  const int kb = step * s.nb;
  const int w = min(s.nb, (int)f.ns - kb);
  const gdbl* D = f.L + (int64_t)kb * M + kb;
  {
    double v[16];   // all 16 loads in flight before the LDS stores
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int idx = threadIdx.x + 256 * u, i = idx & 63, j = idx >> 6;
      v[u] = (i < w && j < w) ? D[(int64_t)j * M + i] : (i == j ? 1.0 : 0.0);
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int idx = threadIdx.x + 256 * u, i = idx & 63, j = idx >> 6;
      sD[j * 65 + i] = v[u];
    }
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const bool upper = part >= 4;
  const int c0 = ((part & 3) * 4 + wv) * 4;   // this wave's columns c0 .. c0+3
  double z[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) z[r] = lane == c0 + r ? 1.0 : 0.0;
  double* out = tinv + slot * 8192 + (upper ? 4096 : 0);
  if (!upper) {
    // L z = e_c: z_j is final at step j; rows i > j subtract L[i][j] z_j
#pragma unroll 4
    for (int j = 0; j < 63; ++j) {
      const double lij = sD[j * 65 + lane];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const double zj = readlane_f64(z[r], j);
        if (lane > j) z[r] = fma(-lij, zj, z[r]);
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) out[(int64_t)(c0 + r) * 64 + lane] = lane > c0 + r ? -z[r] : 0.0;
  } else {
    // U y = e_c: y_j is final at step j after its division; rows i < j subtract U[i][j] y_j
    const double rd = recip(sD[lane * 65 + lane]);
#pragma unroll 4
    for (int j = 63; j >= 0; --j) {
      const double uij = sD[j * 65 + lane];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (lane == j) z[r] *= rd;
        const double yj = readlane_f64(z[r], j);
        if (lane < j) z[r] = fma(-uij, yj, z[r]);
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int c = c0 + r;
      out[(int64_t)c * 64 + lane] = lane == c ? 1.0 - z[r] : (lane < c ? -z[r] : 0.0);
    }
  }
}

#ifdef SMLU_CLOCK_PROBE
// arm != 0: zero the counters and arm the probe; arm == 0: copy the 8 counters out and disarm
extern "C" int smlu_dev_gemm_clock(int arm, unsigned long long* out) {
  static unsigned long long* buf = nullptr;
  if (!buf && hipMalloc(&buf, 8 * sizeof(unsigned long long)) != hipSuccess) return -1;
  unsigned long long* p = nullptr;
  if (arm) {
    if (hipMemset(buf, 0, 8 * sizeof(unsigned long long)) != hipSuccess) return -1;
    p = buf;
  } else {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (out && hipMemcpy(out, buf, 8 * sizeof(unsigned long long), hipMemcpyDeviceToHost) != hipSuccess) return -1;
  }
  return hipMemcpyToSymbol(HIP_SYMBOL(g_clock_probe), &p, sizeof p) == hipSuccess ? 0 : -1;
}
#endif

// ------------------------------------------------------------------------------------
// Host-side launch wrappers (called from smlu.cpp)
// ------------------------------------------------------------------------------------
hipError_t launch_gemm_g(hipStream_t st, int64_t ntiles, const GemmTask* tasks, int ntask, int tile,
                         int64_t maxwg, int32_t* info, double* growth, double piv_tol) {
  if (ntiles <= 0) return hipSuccess;
  const GrowthArgs ga{info, growth, piv_tol};
  const bool trsm = info != nullptr;
  if (tile == 135 && trsm) k_gemm128_mfma3<true, true><<<(unsigned)ntiles, 256, 0, st>>>(tasks, ntask, ga);
  else if (tile == 135) k_gemm128_mfma3<false, true><<<(unsigned)ntiles, 256, 0, st>>>(tasks, ntask, ga);
  else if (tile == 131 && trsm) k_gemm128_mfma3<true><<<(unsigned)ntiles, 256, 0, st>>>(tasks, ntask, ga);
  else if (tile == 131) k_gemm128_mfma3<false><<<(unsigned)ntiles, 256, 0, st>>>(tasks, ntask, ga);
  else if (tile == 65 && trsm) k_gemm_k64<true><<<(unsigned)ntiles, 256, 0, st>>>(tasks, ntask, ga);
  else if (tile == 65) k_gemm_k64<false><<<(unsigned)ntiles, 256, 0, st>>>(tasks, ntask, ga);
  else if (tile == 66 && trsm) k_gemm64_mfma<true><<<(unsigned)ntiles, 256, 0, st>>>(tasks, ntask, ga);
  else if (tile == 66) k_gemm64_mfma<false><<<(unsigned)ntiles, 256, 0, st>>>(tasks, ntask, ga);
  else if (trsm) k_gemm<true><<<(unsigned)ntiles, 256, 0, st>>>(tasks, ntask, ga);
  else k_gemm<false><<<(unsigned)ntiles, 256, 0, st>>>(tasks, ntask, ga);
  return hipGetLastError();
}
hipError_t launch_gemm(hipStream_t st, int64_t ntiles, const GemmTask* tasks, int ntask, int tile,
                       int64_t maxwg) {
  return launch_gemm_g(st, ntiles, tasks, ntask, tile, maxwg, nullptr, nullptr, 1.0);
}
hipError_t launch_urows(hipStream_t st, int cnt, const URowTask* tasks, const SNode* sn, double* store,
                        const double* tinv) {
  if (cnt <= 0) return hipSuccess;
  k_urows<<<(unsigned)cnt, 256, 0, st>>>(tasks, sn, store, tinv);   // OB <= 384 (QMAX): checked by the caller
  return hipGetLastError();
}
hipError_t launch_tri_inv(hipStream_t st, int cnt, int step, const int32_t* list, const SNode* sn,
                          double* store, double* scratch, double* tinv) {
  if (cnt <= 0) return hipSuccess;
  k_tri_inv<<<(unsigned)cnt * 8, 256, 0, st>>>(list, step, sn, store, scratch, tinv);
  return hipGetLastError();
}

}  // namespace smlu
