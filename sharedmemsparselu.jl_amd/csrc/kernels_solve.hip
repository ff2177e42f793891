// kernels_solve.hip — level-scheduled forward/backward solves (lsolve!/rsolve!, src/SharedMemSparseLU.jl:349-392)
// and ldiv!'s scale/permute steps (:318-339).
#include <climits>

#include "kernels_common.hpp"

namespace smlu {

// ------------------------------------------------------------------------------------
// Solves.  Front vectors v_s (M doubles) live in vbuf[voff[s]].
// Forward (L): gather own rows + children's update vectors, apply the front's row
// permutation, unit-lower solve of the diagonal block in 64-column blocks (one wave does
// the block by shuffles, all waves apply the block to the rows below), leave
// v[ns:M) = update vector for the parent.
// ------------------------------------------------------------------------------------
// Small-front solves (one workgroup per front): the bw x bw diagonal block is staged in LDS by
// all 256 threads (coalesced), then one wave runs the shuffle-free chain from LDS.
__device__ __forceinline__ void stage_block(double* __restrict__ sD, const double* __restrict__ D,
                                            int64_t M, int bw, int tid) {
  for (int idx = tid; idx < bw * 64; idx += 256) {
    const int i = idx & 63, j = idx >> 6;
    if (i < bw) sD[j * 65 + i] = D[(int64_t)j * M + i];
  }
}
// Branch-free chain: every lane computes the update and keeps it by a select (no exec-mask changes
// per step); the upper solve's reciprocal of lane j's pivot is computed before the chain.  Same
// values as the guarded loop (the selected operation is the same fma / multiply), bitwise.
template <bool UPPER>
__device__ __forceinline__ double tri_lds(double xi, const double* __restrict__ sD, int bw, int lane) {
  if (!UPPER) {
    for (int j = 0; j < bw; ++j) {
      const double t = fma(-sD[j * 65 + lane], readlane_f64(xi, j), xi);
      xi = (lane > j && lane < bw) ? t : xi;
    }
  } else {
    const double dinv = lane < bw ? recip(sD[lane * 65 + lane]) : 1.0;
    for (int j = bw - 1; j >= 0; --j) {
      xi = lane == j ? xi * dinv : xi;
      const double t = fma(-sD[j * 65 + lane], readlane_f64(xi, j), xi);
      xi = lane < j ? t : xi;
    }
  }
  return xi;
}

// Multi-RHS: every solve kernel takes `rh` (rh.n right-hand sides, column r of x at
// x + r*rh.ldx, of the front vectors at vbuf + r*rh.ldv) and is instantiated for a batch width
// NR >= rh.n (1, 4, 8, 16).  Element-wise loops run over (rhs, row) pairs flattened into one
// index space (one memory round trip for all right-hand sides, not one per rhs); every factor
// value loaded from HBM is applied to all right-hand sides; read-modify-writes of the front
// vectors load all right-hand sides before the first store.  With NR == 1 the arithmetic and its
// order are those of the single-vector solve.
constexpr int kMaxRhs = kMultiRhs;

// st(r, i, ld(r, i)) for r < nr, i < cnt, strided over the workgroup's nthr threads, four
// (r, i) pairs per thread and round: the four loads are issued before the first store (the
// pairs are distinct, so the stores never feed the loads of the same round).  cnt * nr < 2^31.
template <int NR, class LD, class ST>
__device__ __forceinline__ void map_ri(int nr, int64_t cnt, int tid, int nthr, LD&& ld, ST&& st) {
  constexpr int U = 4;
  const uint32_t c = (uint32_t)cnt, tot = c * (uint32_t)(NR == 1 ? 1 : nr);
  for (uint32_t base = tid; base < tot; base += U * nthr) {
    double val[U];
    uint32_t rr[U], ii[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t e = base + u * nthr;
      rr[u] = NR == 1 ? 0 : e / c;
      ii[u] = e - rr[u] * c;
      val[u] = e < tot ? ld((int)rr[u], (int64_t)ii[u]) : 0.0;
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (base + u * nthr < tot) st((int)rr[u], (int64_t)ii[u], val[u]);
  }
}

// Front vector = own rows of x + children's update vectors; the diagonal block's rows permuted
// into x (the front's pivot order) and back into v.  Shared by the small-front and big-front
// forward kernels.
template <int NR>
__device__ __forceinline__ void fwd_gather_front(const SNode& s, const SNode* __restrict__ sn,
                                                 const int32_t* __restrict__ chlist,
                                                 const int32_t* __restrict__ relmap,
                                                 const int32_t* __restrict__ rowperm, double* __restrict__ x,
                                                 double* __restrict__ vbuf, const Rhs& rh, int nr, int tid) {
  const int64_t M = (int64_t)s.ns + s.nu, ns = s.ns;
  map_ri<NR>(nr, M, tid, 256, [&](int r, int64_t i) { return i < ns ? x[r * rh.ldx + s.first + i] : 0.0; },
             [&](int r, int64_t i, double val) { vbuf[r * rh.ldv + s.voff + i] = val; });
  __syncthreads();
  for (int c = s.chbeg; c < s.chend; ++c) {
    const SNode ch = sn[chlist[c]];
    const int32_t* rm = relmap + ch.rowptr;
    // parent += child: both operands loaded per round (a child's relmap rows are distinct)
    map_ri<NR>(nr, ch.nu, tid, 256,
               [&](int r, int64_t i) {
                 return vbuf[r * rh.ldv + s.voff + rm[i]] + vbuf[r * rh.ldv + ch.voff + ch.ns + i];
               },
               [&](int r, int64_t i, double val) { vbuf[r * rh.ldv + s.voff + rm[i]] = val; });
    __syncthreads();
  }
  map_ri<NR>(nr, ns, tid, 256, [&](int r, int64_t i) { return vbuf[r * rh.ldv + s.voff + rowperm[s.first + i]]; },
             [&](int r, int64_t i, double val) { x[r * rh.ldx + s.first + i] = val; });
  __syncthreads();
  map_ri<NR>(nr, ns, tid, 256, [&](int r, int64_t i) { return x[r * rh.ldx + s.first + i]; },
             [&](int r, int64_t i, double val) { vbuf[r * rh.ldv + s.voff + i] = val; });
}

// v[i] -= sum_{j < bw} D[j*M + i] * xs[j][r] for every rhs r, rows i in [lo, hi): the old values
// of all right-hand sides are loaded before the slab loop, stored after it.
template <int NR>
__device__ __forceinline__ void apply_block(const double* __restrict__ D, int64_t M, int bw, int64_t lo,
                                            int64_t hi, const double (*xs)[NR], double* __restrict__ v,
                                            const Rhs& rh, int nr, int tid) {
  for (int64_t i = lo + tid; i < hi; i += 256) {
    double acc[NR], o[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      acc[r] = 0.0;
      o[r] = r < nr ? v[r * rh.ldv + i] : 0.0;
    }
#pragma unroll 1
    for (int h = 0; h < 64; h += 32) {   // 32 slab values per memory round trip
      double d[32];
#pragma unroll
      for (int j = 0; j < 32; ++j) d[j] = h + j < bw ? D[(h + j) * M + i] : 0.0;
#pragma unroll
      for (int j = 0; j < 32; ++j) {
        if (h + j < bw) {
#pragma unroll
          for (int r = 0; r < NR; ++r)
            if (r < nr) acc[r] = fma(d[j], xs[h + j][r], acc[r]);
        }
      }
    }
#pragma unroll
    for (int r = 0; r < NR; ++r)
      if (r < nr) v[r * rh.ldv + i] = o[r] - acc[r];
  }
}

// Diagonal 64x64 block (staged in sD) solved for every rhs: waves take right-hand sides
// round-robin; result into xs and v.
template <bool UPPER, int NR>
__device__ __forceinline__ void solve_block_lds(const double* __restrict__ sD, int64_t jb, int bw,
                                                double (*xs)[NR], double* __restrict__ v, const Rhs& rh,
                                                int nr, int lane, int wv) {
  for (int r = wv; r < nr; r += 4) {
    double* vr = v + r * rh.ldv;
    double xi = lane < bw ? vr[jb + lane] : 0.0;
    xi = tri_lds<UPPER>(xi, sD, bw, lane);
    if (lane < bw) {
      xs[lane][r] = xi;
      vr[jb + lane] = xi;
    }
  }
}

template <int NR>
__global__ __launch_bounds__(256) void k_fwd_front(const int32_t* __restrict__ list,
                                                   const SNode* __restrict__ sn,
                                                   const int32_t* __restrict__ chlist,
                                                   const int32_t* __restrict__ relmap,
                                                   const int32_t* __restrict__ rowperm,
                                                   const double* __restrict__ store,
                                                   double* __restrict__ x,
                                                   double* __restrict__ vbuf, Rhs rh) {
  __shared__ double xs[64][NR];   // solved block, right-hand sides contiguous per column
  __shared__ double sD[64 * 65];
  const SNode s = sn[list[blockIdx.x]];
  const int64_t M = (int64_t)s.ns + s.nu, ns = s.ns;
  const int nr = NR == 1 ? 1 : rh.n;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  fwd_gather_front<NR>(s, sn, chlist, relmap, rowperm, x, vbuf, rh, nr, tid);
  __syncthreads();
  const double* Lp = store + s.Loff;
  double* v = vbuf + s.voff;
  for (int64_t jb = 0; jb < ns; jb += 64) {
    const int bw = (int)min<int64_t>(64, ns - jb);
    stage_block(sD, Lp + jb * M + jb, M, bw, tid);
    __syncthreads();
    solve_block_lds<false, NR>(sD, jb, bw, xs, v, rh, nr, lane, wv);
    __syncthreads();
    apply_block<NR>(Lp + jb * M, M, bw, jb + bw, M, xs, v, rh, nr, tid);
    __syncthreads();
  }
  map_ri<NR>(nr, ns, tid, 256, [&](int r, int64_t i) { return vbuf[r * rh.ldv + s.voff + i]; },
             [&](int r, int64_t i, double val) { x[r * rh.ldx + s.first + i] = val; });
}

// Backward (U): x_s -= U12 * x[R_s]; then upper solve of the diagonal block from the bottom.
template <int NR>
__global__ __launch_bounds__(256) void k_bwd_front(const int32_t* __restrict__ list,
                                                   const SNode* __restrict__ sn,
                                                   const int32_t* __restrict__ rows,
                                                   const double* __restrict__ store,
                                                   double* __restrict__ x,
                                                   double* __restrict__ vbuf, Rhs rh) {
  __shared__ double xs[64][NR];   // solved block, right-hand sides contiguous per column
  __shared__ double sD[64 * 65];
  const SNode s = sn[list[blockIdx.x]];
  const int64_t M = (int64_t)s.ns + s.nu, ns = s.ns, nu = s.nu;
  const int nr = NR == 1 ? 1 : rh.n;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int32_t* R = rows + s.rowptr;
  // x_s -= U12 x[R]: x[R] staged through LDS 64 columns at a time (xs doubles as the buffer)
  const double* U12 = store + s.Uoff;
  for (int64_t i0 = 0; i0 < ns; i0 += 256) {
    const int64_t i = i0 + tid;
    double acc[NR], o[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      acc[r] = 0.0;
      o[r] = (i < ns && r < nr) ? x[r * rh.ldx + s.first + i] : 0.0;
    }
    for (int64_t jc = 0; jc < nu; jc += 64) {
      const int cnt = (int)min<int64_t>(64, nu - jc);
      __syncthreads();
      map_ri<NR>(nr, cnt, tid, 256, [&](int r, int64_t j) { return x[r * rh.ldx + R[jc + j]]; },
                 [&](int r, int64_t j, double val) { xs[j][r] = val; });
      __syncthreads();
      if (i < ns) {
#pragma unroll 1
        for (int h = 0; h < 64; h += 32) {   // 32 U12 values per memory round trip
          double u[32];
#pragma unroll
          for (int j = 0; j < 32; ++j) u[j] = h + j < cnt ? U12[(jc + h + j) * ns + i] : 0.0;
#pragma unroll
          for (int j = 0; j < 32; ++j) {
            if (h + j < cnt) {
#pragma unroll
              for (int r = 0; r < NR; ++r)
                if (r < nr) acc[r] = fma(u[j], xs[h + j][r], acc[r]);
            }
          }
        }
      }
    }
    if (i < ns) {
#pragma unroll
      for (int r = 0; r < NR; ++r)
        if (r < nr) vbuf[r * rh.ldv + s.voff + i] = o[r] - acc[r];
    }
  }
  __syncthreads();   // xs is reused by the diagonal sweep below
  const double* Lp = store + s.Loff;  // U11 in the upper triangle of the L panel
  double* v = vbuf + s.voff;
  for (int64_t jb = ((ns - 1) / 64) * 64; jb >= 0; jb -= 64) {
    const int bw = (int)min<int64_t>(64, ns - jb);
    stage_block(sD, Lp + jb * M + jb, M, bw, tid);
    __syncthreads();
    solve_block_lds<true, NR>(sD, jb, bw, xs, v, rh, nr, lane, wv);
    __syncthreads();
    apply_block<NR>(Lp + jb * M, M, bw, 0, jb, xs, v, rh, nr, tid);
    __syncthreads();
  }
  map_ri<NR>(nr, ns, tid, 256, [&](int r, int64_t i) { return vbuf[r * rh.ldv + s.voff + i]; },
             [&](int r, int64_t i, double val) { x[r * rh.ldx + s.first + i] = val; });
}

// Tiny fronts (M <= 128 rows, ns <= 64 pivots: the leaves of the assembly tree -- 257k fronts of
// M = 7 at 128^3 -- and most of the next four levels): one wave per front, four fronts per
// workgroup, lane i owns rows i and i + 64 of the front -- no workgroup barriers, the factor rows
// are loaded once into registers and applied to every right-hand side.  Same operations in the
// same order as k_fwd_front / k_bwd_front (bitwise identical): forward, the pivot rows run the
// unit-lower chain and the update rows accumulate sum_j L[i,j] x_j then subtract it; backward,
// x_s - U12 x[R] (columns in order, 64 at a time) then the upper chain.
template <int NR>
__global__ __launch_bounds__(256) void k_fwd_tiny(const int32_t* __restrict__ list, int cnt,
                                                  const SNode* __restrict__ sn, const int32_t* __restrict__ chlist,
                                                  const int32_t* __restrict__ relmap,
                                                  const int32_t* __restrict__ rowperm,
                                                  const double* __restrict__ store, double* __restrict__ x,
                                                  double* __restrict__ vbuf, Rhs rh) {
  __shared__ double sv[4][128];
  __shared__ double sx[4][NR][64];   // solved pivot values, for rows 64..127
  __shared__ double s2[4][NR][64];   // gathered values of rows 64..127
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t f = (int64_t)blockIdx.x * 4 + wv;
  if (f >= cnt) return;   // the whole wave: no workgroup barriers below
  const SNode s = sn[list[f]];
  const int ns = s.ns, M = ns + s.nu;
  const int nr = NR == 1 ? 1 : rh.n;
  const double* Lp = store + s.Loff;
  {
    double l[64];
#pragma unroll
    for (int j = 0; j < 64; ++j) l[j] = (lane < M && j < ns) ? Lp[(int64_t)j * M + lane] : 0.0;
    const int pr = lane < ns ? rowperm[s.first + lane] : lane;
    for (int r = 0; r < nr; ++r) {
      double* xr = x + r * rh.ldx;
      double* vr = vbuf + r * rh.ldv;
      sv[wv][lane] = lane < ns ? xr[s.first + lane] : 0.0;
      sv[wv][64 + lane] = 0.0;
      wave_lds_sync();
      for (int c = s.chbeg; c < s.chend; ++c) {   // parent += child, children in order
        const SNode ch = sn[chlist[c]];
        for (int q = lane; q < ch.nu; q += 64) {   // a child's target rows are distinct
          const int t = relmap[ch.rowptr + q];
          sv[wv][t] = sv[wv][t] + vr[ch.voff + ch.ns + q];
        }
        wave_lds_sync();
      }
      double val = lane < M ? sv[wv][pr] : 0.0;   // pivot rows in the front's pivot order
      if (M > 64) s2[wv][r][lane] = 64 + lane < M ? sv[wv][64 + lane] : 0.0;
      wave_lds_sync();                            // every lane read before the next rhs overwrites
      double acc = 0.0;
#pragma unroll
      for (int j = 0; j < 64; ++j) {
        if (j < ns) {
          const double xj = readlane_f64(val, j);
          if (lane > j && lane < ns) val = fma(-l[j], xj, val);
          else if (lane >= ns) acc = fma(l[j], xj, acc);
        }
      }
      if (lane < ns) {
        xr[s.first + lane] = val;
        vr[s.voff + lane] = val;
        if (M > 64) sx[wv][r][lane] = val;
      } else if (lane < M) {
        vr[s.voff + lane] = val - acc;
      }
    }
  }
  if (M <= 64) return;
  wave_lds_sync();
  // rows 64..127 (update rows: ns <= 64): sum_j L[64+lane, j] x_j, then subtract
  double l2[64];
#pragma unroll
  for (int j = 0; j < 64; ++j) l2[j] = (64 + lane < M && j < ns) ? Lp[(int64_t)j * M + 64 + lane] : 0.0;
  for (int r = 0; r < nr; ++r) {
    double acc = 0.0;
#pragma unroll
    for (int j = 0; j < 64; ++j)
      if (j < ns) acc = fma(l2[j], sx[wv][r][j], acc);
    if (64 + lane < M) vbuf[r * rh.ldv + s.voff + 64 + lane] = s2[wv][r][lane] - acc;
  }
}

template <int NR>
__global__ __launch_bounds__(256) void k_bwd_tiny(const int32_t* __restrict__ list, int cnt,
                                                  const SNode* __restrict__ sn, const int32_t* __restrict__ rows,
                                                  const double* __restrict__ store, double* __restrict__ x,
                                                  double* __restrict__ vbuf, Rhs rh) {
  __shared__ double sv[4][NR][64];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t f = (int64_t)blockIdx.x * 4 + wv;
  if (f >= cnt) return;
  const SNode s = sn[list[f]];
  const int ns = s.ns, nu = s.nu;
  const int64_t M = (int64_t)ns + nu;
  const int nr = NR == 1 ? 1 : rh.n;
  {   // x_s - U12 x[R]: U12 row `lane` in registers 64 columns at a time, x[R_j] from lane j
    const double* U12 = store + s.Uoff;
#pragma unroll 1
    for (int jb = 0; jb < nu; jb += 64) {
      __builtin_amdgcn_sched_barrier(0);   // one 64-column slab live at a time
      double u[64];
#pragma unroll
      for (int j = 0; j < 64; ++j) u[j] = (lane < ns && jb + j < nu) ? U12[(int64_t)(jb + j) * ns + lane] : 0.0;
      const int32_t rj = jb + lane < nu ? rows[s.rowptr + jb + lane] : 0;
      for (int r = 0; r < nr; ++r) {
        const double* xr = x + r * rh.ldx;
        const double xR = jb + lane < nu ? xr[rj] : 0.0;
        double acc = jb == 0 ? 0.0 : sv[wv][r][lane];
#pragma unroll
        for (int j = 0; j < 64; ++j) {
          if (jb + j < nu) {
            const double xj = readlane_f64(xR, j);
            acc = fma(u[j], xj, acc);
          }
        }
        sv[wv][r][lane] = acc;
      }
    }
    for (int r = 0; r < nr; ++r) {
      const double o = lane < ns ? x[r * rh.ldx + s.first + lane] : 0.0;
      sv[wv][r][lane] = o - (nu > 0 ? sv[wv][r][lane] : 0.0);
    }
  }
  wave_lds_sync();
  __builtin_amdgcn_sched_barrier(0);   // the U12 slab dies before the U11 rows are loaded
  const double* Lp = store + s.Loff;   // U11 in the upper triangle of the L panel
  double l[64];
#pragma unroll
  for (int j = 0; j < 64; ++j) l[j] = (lane < ns && j < ns) ? Lp[(int64_t)j * M + lane] : 0.0;
  const double dinv = lane < ns ? recip(Lp[(int64_t)lane * M + lane]) : 1.0;
  for (int r = 0; r < nr; ++r) {
    double val = lane < ns ? sv[wv][r][lane] : 0.0;
#pragma unroll
    for (int j = 63; j >= 0; --j) {
      if (j < ns) {
        if (lane == j) val = val * dinv;
        const double xj = readlane_f64(val, j);
        if (lane < j) val = fma(-l[j], xj, val);
      }
    }
    if (lane < ns) {
      x[r * rh.ldx + s.first + lane] = val;
      vbuf[r * rh.ldv + s.voff + lane] = val;
    }
  }
}

// Micro fronts (M <= 8 rows: the 240k leaves of the 128^3 tree are (M, ns) = (7, 1) or (6, 1)),
// one right-hand side: eight fronts per wave, lane group g = lane >> 3 holds front g's rows
// (row i = lane & 7), broadcasts within the group by __shfl.  A wave per front (k_fwd_tiny) left
// 56 of 64 lanes idle and ran at 3 waves/SIMD; these kernels keep ~32 waves per CU in flight.
// Exactly k_fwd_tiny's / k_bwd_tiny's operations in the same order per element (bitwise equal);
// batched solves loop over their right-hand sides here with the factor rows loaded once (round 6:
// they used to take a whole wave per micro front through the tiny kernels).
__global__ __launch_bounds__(256) void k_fwd_micro(const int32_t* __restrict__ list, int cnt,
                                                   const SNode* __restrict__ sn, const int32_t* __restrict__ chlist,
                                                   const int32_t* __restrict__ relmap,
                                                   const int32_t* __restrict__ rowperm,
                                                   const double* __restrict__ store, double* __restrict__ x,
                                                   double* __restrict__ vbuf, Rhs rh) {
  __shared__ double sv[32][8];
  const int lane = threadIdx.x & 63, g = threadIdx.x >> 3, i = threadIdx.x & 7;
  const int64_t f = (int64_t)blockIdx.x * 32 + g;
  const bool act = f < cnt;
  SNode s{};
  if (act) s = sn[list[f]];
  const int ns = act ? s.ns : 0, M = act ? s.ns + s.nu : 0;
  const double* Lp = store + s.Loff;
  double l[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) l[j] = (i < M && j < ns) ? Lp[(int64_t)j * M + i] : 0.0;
  const int pr = i < ns ? rowperm[s.first + i] : i;
  const int gb = lane & ~7;
  for (int r = 0; r < rh.n; ++r) {   // the factor rows loaded once for every right-hand side
    double* xr = x + r * rh.ldx;
    double* vr = vbuf + r * rh.ldv;
    sv[g][i] = i < ns ? xr[s.first + i] : 0.0;
    wave_lds_sync();
    for (int c = act ? s.chbeg : 0; c < (act ? s.chend : 0); ++c) {   // parent += child, children in order
      const SNode ch = sn[chlist[c]];
      for (int q = i; q < ch.nu; q += 8) {
        const int t = relmap[ch.rowptr + q];
        sv[g][t] = sv[g][t] + vr[ch.voff + ch.ns + q];
      }
      wave_lds_sync();
    }
    wave_lds_sync();
    double val = i < M ? sv[g][pr] : 0.0;
    double acc = 0.0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const double xj = __shfl(val, gb + j, 64);
      if (j < ns) {
        if (i > j && i < ns) val = fma(-l[j], xj, val);
        else if (i >= ns) acc = fma(l[j], xj, acc);
      }
    }
    if (i < ns) {
      xr[s.first + i] = val;
      vr[s.voff + i] = val;
    } else if (i < M) {
      vr[s.voff + i] = val - acc;
    }
    wave_lds_sync();   // every lane read sv before the next right-hand side overwrites it
  }
}

__global__ __launch_bounds__(256) void k_bwd_micro(const int32_t* __restrict__ list, int cnt,
                                                   const SNode* __restrict__ sn, const int32_t* __restrict__ rows,
                                                   const double* __restrict__ store, double* __restrict__ x,
                                                   double* __restrict__ vbuf, Rhs rh) {
  const int lane = threadIdx.x & 63, i = threadIdx.x & 7;
  const int64_t f = (int64_t)blockIdx.x * 32 + (threadIdx.x >> 3);
  const bool act = f < cnt;
  SNode s{};
  if (act) s = sn[list[f]];
  const int ns = act ? s.ns : 0, nu = act ? s.nu : 0;
  const int64_t M = (int64_t)ns + nu;
  const double* Lp = store + s.Loff;
  double l[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) l[j] = (i < ns && j < ns) ? Lp[(int64_t)j * M + i] : 0.0;
  const double dinv = i < ns ? recip(Lp[(int64_t)i * M + i]) : 1.0;
  const int gb = lane & ~7;
  for (int r = 0; r < rh.n; ++r) {
    double* xr = x + r * rh.ldx;
    // x_s - U12 x[R] (columns in order), then the upper chain
    double acc = 0.0;
    if (i < ns) {
      const double* U12 = store + s.Uoff;
      for (int j = 0; j < nu; ++j) acc = fma(U12[(int64_t)j * ns + i], xr[rows[s.rowptr + j]], acc);
    }
    const double o = i < ns ? xr[s.first + i] : 0.0;
    double val = o - (nu > 0 ? acc : 0.0);
    if (!(i < ns)) val = 0.0;
#pragma unroll
    for (int j = 7; j >= 0; --j) {
      if (j < ns && i == j) val = val * dinv;
      const double xj = __shfl(val, gb + j, 64);
      if (j < ns && i < j) val = fma(-l[j], xj, val);
    }
    if (i < ns) {
      xr[s.first + i] = val;
      vbuf[r * rh.ldv + s.voff + i] = val;
    }
  }
}

// ------------------------------------------------------------------------------------
// Solves for large fronts (ns > 256): the diagonal block sweep is split over workgroups.
// k_fwd_gather: front vector = own rows + children's update vectors, row permutation.
// k_tri_block (step t): every workgroup re-solves the 64x64 diagonal block from v (read-only in
//   this launch), applies it to its 256-row chunk; chunk 0 publishes the solved block into x.
// k_bwd_u12: x_s -= U12 x[R_s] by row chunks.
// ------------------------------------------------------------------------------------
// One workgroup per (front, right-hand side): blockIdx.y selects the rhs.
__global__ __launch_bounds__(256) void k_fwd_gather(const int32_t* __restrict__ list,
                                                    const SNode* __restrict__ sn,
                                                    const int32_t* __restrict__ chlist,
                                                    const int32_t* __restrict__ relmap,
                                                    const int32_t* __restrict__ rowperm,
                                                    double* __restrict__ x, double* __restrict__ vbuf, Rhs rh) {
  const SNode s = sn[list[blockIdx.x]];
  const int r = blockIdx.y;
  fwd_gather_front<1>(s, sn, chlist, relmap, rowperm, x + r * rh.ldx, vbuf + r * rh.ldv, rh, 1, threadIdx.x);
}

// Large-front gather, one thread per front row i over as many workgroups as the rows need (the
// one-workgroup-per-front k_fwd_gather left a 16k-row root to a single CU): the row's pre-pivoting
// source j = rowperm(i) for pivot rows, itself for update rows; value = own x_j (pivot rows) or 0,
// plus the children's update-vector entries that map to j, in child order -- per element exactly the
// additions of k_fwd_gather (bitwise equal).  Writes v only: x is not touched before the forward
// solve writes every pivot row (the sweep and k_tri_block read v), so no row's original x is
// overwritten while other workgroups read it.  gptr (per front row, offset ft.pad) -> gent (vbuf
// index of each contribution).
template <int NR>
__global__ __launch_bounds__(256) void k_fwd_pull(const FrontTile* __restrict__ ft, int nft, const SNode* __restrict__ sn,
                                                  const int32_t* __restrict__ rowperm, const int32_t* __restrict__ gptr,
                                                  const int32_t* __restrict__ gent, const double* __restrict__ x,
                                                  double* __restrict__ vbuf, Rhs rh) {
  const int64_t b = blockIdx.x;
  const int fi = find_front_tile(ft, nft, b);
  const SNode s = sn[ft[fi].s];
  const int64_t i = (b - ft[fi].wg0) * 256 + threadIdx.x;
  const int64_t M = (int64_t)s.ns + s.nu, ns = s.ns;
  if (i >= M) return;
  const int64_t j = i < ns ? rowperm[s.first + i] : i;
  const int32_t* P = gptr + ft[fi].pad;
  const int32_t p0 = P[j], p1 = P[j + 1];
  const int nr = NR == 1 ? 1 : rh.n;
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    if (r < nr) {
      double val = j < ns ? x[r * rh.ldx + s.first + j] : 0.0;
      for (int32_t p = p0; p < p1; ++p) val = val + vbuf[r * rh.ldv + gent[p]];
      vbuf[r * rh.ldv + s.voff + i] = val;
    }
  }
}

// One 64-column step of a large front: the first CW waves of every workgroup solve the 64x64
// diagonal block for the right-hand sides (tri64, the diagonal block's rows loaded once per wave,
// CW right-hand sides at a time; each workgroup re-solves it, no inter-workgroup hand-off); the
// last four waves own one row each of the workgroup's 256-row chunk and load that row's 64 slab
// values and its old values before the solved block arrives (the memory round trips overlap),
// then apply the block to every right-hand side.  At most two waves per SIMD: d[64] and row[64]
// keep 128 VGPRs live, so allow 256 rather than spill.
template <bool UPPER, int NR>
__global__ __launch_bounds__(NR == 1 ? 320 : 512) __attribute__((amdgpu_waves_per_eu(1, 2)))
void k_tri_block(const FrontTile* __restrict__ ft, int nft, int step, const SNode* __restrict__ sn,
                 const double* __restrict__ store, double* __restrict__ x, double* __restrict__ vbuf, Rhs rh) {
  constexpr int CW = NR == 1 ? 1 : 4;        // chain waves
  constexpr int PR = (NR + CW - 1) / CW;     // right-hand sides per chain wave
  __shared__ double xs[64][NR];
  const int64_t b = blockIdx.x;
  const int fi = find_front_tile(ft, nft, b);
  const SNode s = sn[ft[fi].s];
  const int64_t chunk = b - ft[fi].wg0;
  const int64_t M = (int64_t)s.ns + s.nu, ns = s.ns;
  const int64_t nblk = (ns + 63) / 64;
  const int64_t jb = UPPER ? (nblk - 1 - step) * 64 : (int64_t)step * 64;
  const int bw = (int)min<int64_t>(64, ns - jb);
  const int nr = NR == 1 ? 1 : rh.n;
  const double* Lp = store + s.Loff;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (wv < CW) {
    double xi[PR];
#pragma unroll
    for (int k = 0; k < PR; ++k) {
      const int r = wv + k * CW;
      xi[k] = (r < nr && lane < bw) ? vbuf[r * rh.ldv + s.voff + jb + lane] : 0.0;
    }
    double row[64];   // the diagonal block's row `lane`, loaded once for all right-hand sides
    load_tri_row64<UPPER>(row, Lp + jb * M + jb, M, bw, lane);
    const double dinv = UPPER ? diag_recip(Lp + jb * M + jb, M, bw, lane) : 1.0;
    if (UPPER) tri64_scale_upper(row, dinv, bw);
#pragma unroll
    for (int k = 0; k < PR; ++k) {
      const int r = wv + k * CW;
      if (r < nr) {
        const double y = tri64_row<UPPER>(xi[k], row, dinv, bw);
        if (lane < bw) {
          xs[lane][r] = y;
          if (chunk == 0) x[r * rh.ldx + s.first + jb + lane] = y;
        }
      }
    }
    __syncthreads();
    return;
  }
  // rows updated by this chunk: forward -> [jb+bw, M), backward -> [0, jb)
  const int64_t r0 = UPPER ? chunk * 256 : jb + bw + chunk * 256;
  const int64_t r1 = UPPER ? jb : M;
  const int64_t i = r0 + tid - 64 * CW;
  const bool has = i < r1;
  double d[64], o[NR];
#pragma unroll
  for (int j = 0; j < 64; ++j) d[j] = (has && j < bw) ? Lp[(jb + j) * M + i] : 0.0;
#pragma unroll
  for (int r = 0; r < NR; ++r) o[r] = (has && r < nr) ? vbuf[r * rh.ldv + s.voff + i] : 0.0;
  __syncthreads();
  if (has) {
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      if (r < nr) {
        const double acc = dot64_split(d, bw, [&](int j) { return xs[j][r]; });
        vbuf[r * rh.ldv + s.voff + i] = o[r] - acc;
      }
    }
  }
}

// ------------------------------------------------------------------------------------
// Sync-free triangular sweep of the large fronts of one level (one launch per level and direction,
// replacing one launch per 64-column block).  Work item = a chunk of 256 rows (forward: rows
// [256q, 256q+256) of the front; backward: the pivot blocks nblk-1-4q-t, t < 4); one workgroup,
// one thread per row.  A chunk applies the column blocks solved by earlier chunks of its front as
// they are published, then runs its own (up to four) diagonal blocks in sequence inside the
// workgroup -- wave t solves block 4q+t (the 64-step readlane chain of tri64_row), the waves below
// apply it -- and publishes each solved block.
// Protocol: every word shared between workgroups is accessed by device-scope ATOMICS, performed at
// the memory side, so no cache level can hand out a stale copy and nothing has to be reset between
// solves (a hipGraph replay of reset + sweep does not guarantee that other XCDs' L2s see the reset:
// a single-vector solve after a batched one read stale flags and hung).
//  * tickets: one 64-bit counter per launch, never reset; a workgroup's ticket t gives its work item
//    t mod nwg and the launch's epoch t / nwg + 1 (launches of a sweep are stream-ordered, so each
//    takes one contiguous range of tickets);
//  * block b is published by writing its 64 x NR solved values into its hand-off slot (atomic swaps)
//    and then setting flag[b] to the epoch (atomic max) behind the wave's vmcnt drain and a barrier;
//  * a consumer polls flag[b] (atomic compare-and-swap that never matches) until it reaches the epoch
//    and reads the slot the same way on the raw bits.
// Deadlock-free: items are taken in ticket order and an item only waits on items of lower tickets
// (earlier chunks of the same front), which are running.  Per right-hand side the arithmetic does
// not depend on the batch width (a batched column is bitwise the single solve).
// tick: this launch's counter; flags of front f at flags + pad_f; hand-off slot of flag g at
// xh + g * 64 * kMultiRhs.  status: set to 1 if a wait ever times out (never expected).
// ------------------------------------------------------------------------------------
// Reads as compare-and-swap with a value never stored (an idempotent add of 0 would be lowered to
// a plain cached load): the returned old value comes from the memory-side atomic unit.
__device__ __forceinline__ int32_t atomic_read_i32(int32_t* p) {
  int32_t e = INT32_MIN;   // flags hold epochs >= 0
  __hip_atomic_compare_exchange_strong(p, &e, INT32_MIN, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
  return e;
}
__device__ __forceinline__ double atomic_read_f64(double* p) {
  unsigned long long e = 0x7ff4dead5eed0001ull;   // a signalling-NaN pattern no solve writes
  __hip_atomic_compare_exchange_strong(reinterpret_cast<unsigned long long*>(p), &e, 0x7ff4dead5eed0001ull,
                                       __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return __longlong_as_double((long long)e);
}
__device__ __forceinline__ void atomic_write_f64(double* p, double v) {
  (void)__hip_atomic_exchange(reinterpret_cast<unsigned long long*>(p), (unsigned long long)__double_as_longlong(v),
                              __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Bounded wait for flag f to reach the epoch.  A wait that gives up raises *status; the host reads
// it after every solve and re-runs the solve on the per-block schedule (smlu.cpp: run_solve_dev), so
// a timed-out chunk's values are never returned.  spin <= 0 reports every wait as timed out (the
// tests' forced-fallback knob SMLU_SWEEP_SPIN=0).
__device__ __forceinline__ void sweep_wait(int32_t* f, int32_t epoch, int32_t* status, int spin) {
  if (threadIdx.x == 0) {
    if (spin <= 0) {
      (void)__hip_atomic_fetch_max(status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      int n = 0;
      while (atomic_read_i32(f) < epoch) {
        __builtin_amdgcn_s_sleep(1);
        if (++n > spin) {
          (void)__hip_atomic_fetch_max(status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
    }
  }
  __syncthreads();
}

// Dev instrumentation (tools/sweep_trace.py): one launch shape (grid, direction) records per work item
// and wave the 100 MHz real-time clock at its start, after its external blocks, before and after its
// own substitution, after publishing, and at its end.  Compiled in with -DSMLU_SWEEP_TRACE only
// (make CXXFLAGS+=-DSMLU_SWEEP_TRACE); the product build has neither the buffer nor the hook.
#ifdef SMLU_SWEEP_TRACE
struct SweepTrace {
  long long* buf;
  int nwg, upper;
};
__device__ SweepTrace g_sweep_trace;
__device__ __forceinline__ void sweep_mark(bool upper, int64_t item, int wv, int k) {
  const SweepTrace t = g_sweep_trace;
  if (t.buf && (int)gridDim.x == t.nwg && (int)upper == t.upper && (threadIdx.x & 63) == 0)
    t.buf[(item * kSweepWK + wv) * 8 + k] = (long long)__builtin_amdgcn_s_memrealtime();
}
#else
__device__ __forceinline__ void sweep_mark(bool, int64_t, int, int) {}
#endif

template <bool UPPER, int NR>
__global__ __launch_bounds__(64 * kSweepWK) __attribute__((amdgpu_waves_per_eu(1, (kSweepWK + 3) / 4)))
void k_tri_sweep(const FrontTile* __restrict__ ft, int nft, unsigned long long* __restrict__ tick,
                 int32_t* __restrict__ flags0, double* __restrict__ xh, int32_t* __restrict__ status,
                 const SNode* __restrict__ sn, const double* __restrict__ store, double* __restrict__ x,
                 double* __restrict__ vbuf, Rhs rh, int spin) {
  __shared__ double xs[64][NR];
  __shared__ unsigned long long s_ticket;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (tid == 0) s_ticket = __hip_atomic_fetch_add(tick, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const int64_t item = (int64_t)(s_ticket % gridDim.x);
  const int32_t epoch = (int32_t)(s_ticket / gridDim.x) + 1;
  sweep_mark(UPPER, item, wv, 0);
  const int fi = find_front_tile(ft, nft, item);
  const SNode s = sn[ft[fi].s];
  int32_t* flags = flags0 + ft[fi].pad;
  double* xhf = xh + (int64_t)ft[fi].pad * 64 * kMultiRhs;   // hand-off slots of this front's blocks
  const int64_t q = item - ft[fi].wg0;
  const int64_t M = (int64_t)s.ns + s.nu, ns = s.ns, nblk = (ns + 63) / 64;
  const double* Lp = store + s.Loff;
  const int nr = NR == 1 ? 1 : rh.n;
  double* v = vbuf + s.voff;
  double* xf = x + s.first;
  // my row; blocks of other chunks (external) and of this chunk (internal, block ids in order)
  int64_t row, myblk;
  if (!UPPER) {
    row = 64 * kSweepWK * q + tid;
    myblk = row < ns ? row / 64 : nblk;
  } else {
    myblk = nblk - 1 - kSweepWK * q - wv;
    row = 64 * myblk + lane;
  }
  const bool has = UPPER ? (myblk >= 0 && row < ns) : row < M;
  double o[NR];
#pragma unroll
  for (int r = 0; r < NR; ++r) o[r] = (has && r < nr) ? v[r * rh.ldv + row] : 0.0;
  // the diagonal block's row of a pivot row, loaded up front (off the chain's critical path)
  double drow[64];
  double dinv = 1.0;
  {
    const bool piv = has && myblk < nblk;
    const int64_t b = piv ? myblk : 0;
    const int bw = (int)min<int64_t>(64, ns - 64 * b);
    const int li = (int)(row - 64 * b);
#pragma unroll
    for (int j = 0; j < 64; ++j)
      drow[j] = (piv && j < bw && (UPPER ? j > li : j < li)) ? Lp[(64 * b + j) * M + row] : 0.0;
    if (UPPER && piv) dinv = recip(Lp[(64 * b + li) * M + row]);
    if (UPPER) tri64_scale_upper(drow, dinv, bw);
  }
  double d[64];   // my row of the column block being applied, loaded before its x is available
  auto load_tile = [&](int64_t c, int bw) {
#pragma unroll
    for (int j = 0; j < 64; ++j) d[j] = j < bw ? Lp[(64 * c + j) * M + row] : 0.0;
  };
  auto fma_tile = [&](int bw) {   // o -= L[row, block] * x_block (x in xs), k_tri_block's dot64_split
#pragma unroll
    for (int r = 0; r < NR; ++r)
      if (r < nr) o[r] -= dot64_split(d, bw, [&](int j) { return xs[j][r]; });
  };
  // external blocks (solved by earlier chunks): forward 0 .. min(WK q, nblk)-1, backward nblk-1
  // down to nblk-WK q (WK = kSweepWK waves, one 64-row block each); every row of this chunk lies beyond them
  const int64_t next = min<int64_t>(kSweepWK * q, nblk);
  for (int64_t e = 0; e < next; ++e) {
    const int64_t c = UPPER ? nblk - 1 - e : e;
    const int bw = (int)min<int64_t>(64, ns - 64 * c);
    if (has) load_tile(c, bw);
    sweep_wait(flags + c, epoch, status, spin);
    if (wv == 0)
      for (int r = 0; r < min(nr, NR); ++r) xs[lane][r] = atomic_read_f64(xhf + (c * kMultiRhs + r) * 64 + lane);
    __syncthreads();
    if (has) fma_tile(bw);
    __syncthreads();
  }
  sweep_mark(UPPER, item, wv, 1);
  // internal blocks: wave t solves block b and publishes it, the waves beyond apply it
  for (int t = 0; t < kSweepWK; ++t) {
    const int64_t b = UPPER ? nblk - 1 - kSweepWK * q - t : kSweepWK * q + t;
    if (b < 0 || b >= nblk) break;
    const int bw = (int)min<int64_t>(64, ns - 64 * b);
    // rows that apply block b: the waves beyond t, and the update rows of wave t when block b is
    // the last, partial one (forward): same per-block arithmetic as every other row
    const bool applies = has && (wv > t || (wv == t && myblk >= nblk));
    if (applies) load_tile(b, bw);
    if (wv == t) {
      sweep_mark(UPPER, item, wv, 2);
      double y[NR];   // the NR chains interleaved (tri64_rows; per column bitwise tri64_row)
#pragma unroll
      for (int r = 0; r < NR; ++r) y[r] = o[r];
      tri64_rows<UPPER, NR>(y, drow, dinv, bw);
      const bool mine = lane < bw && has;
#pragma unroll
      for (int r = 0; r < NR; ++r) {
        if (r < nr) {
          if (mine) o[r] = y[r];
          atomic_write_f64(xhf + (b * kMultiRhs + r) * 64 + lane, mine ? y[r] : 0.0);
          if (mine) {
            xs[lane][r] = y[r];
            xf[r * rh.ldx + 64 * b + lane] = y[r];
            v[r * rh.ldv + 64 * b + lane] = y[r];
          }
        }
      }
      sweep_mark(UPPER, item, wv, 3);
    }
    __syncthreads();   // xs (LDS) visible to the waves that apply block b
    if (wv == t) {
      // publish: raise the flag once this wave's slot writes have completed (vmcnt counts every
      // lane's atomics of the wave); the other waves apply the block meanwhile, so the write
      // round trip is off the chunk's own chain
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) (void)__hip_atomic_fetch_max(flags + b, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (lane == 0) sweep_mark(UPPER, item, t, 4);
    }
    if (applies) fma_tile(bw);
    __syncthreads();
  }
  sweep_mark(UPPER, item, wv, 5);
  // forward: the update rows leave their value for the parent
  if (!UPPER && has && myblk >= nblk) {
#pragma unroll
    for (int r = 0; r < NR; ++r)
      if (r < nr) v[r * rh.ldv + row] = o[r];
  }
}

// x_s[i] (in v) = x[first+i] - sum_j U12[i,j] * x[R_j]: 64 rows per workgroup, 8 waves; wave w
// sums the columns [w*nu/8, (w+1)*nu/8) 32 at a time, the 32 U12 loads of a chunk issued
// together (8 waves x 32 x 512 B in flight per workgroup), x[R] staged per chunk in LDS; the
// eight partial sums are combined in wave order; each U12 value is applied to every rhs.
template <int NR>
__global__ __launch_bounds__(512) void k_bwd_u12(const FrontTile* __restrict__ ft, int nft,
                                                 const SNode* __restrict__ sn,
                                                 const int32_t* __restrict__ rows,
                                                 const double* __restrict__ store,
                                                 const double* __restrict__ x,
                                                 double* __restrict__ vbuf, Rhs rh) {
  constexpr int W = 8, JC = 32;
  __shared__ double xr[W][JC][NR];
  __shared__ double part[W][NR][64];
  const int64_t b = blockIdx.x;
  const int fi = find_front_tile(ft, nft, b);
  const SNode s = sn[ft[fi].s];
  const int64_t chunk = b - ft[fi].wg0;
  const int64_t ns = s.ns, nu = s.nu;
  const int nr = NR == 1 ? 1 : rh.n;
  const int32_t* R = rows + s.rowptr;
  const double* U12 = store + s.Uoff;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int64_t i = chunk * 64 + lane;
  const int64_t j0 = nu * wv / W, j1 = nu * (wv + 1) / W;
  double acc[NR];
#pragma unroll
  for (int r = 0; r < NR; ++r) acc[r] = 0.0;
  for (int64_t jc = j0; jc < j1; jc += JC) {
    const int cnt = (int)min<int64_t>(JC, j1 - jc);
    for (int e = lane; e < cnt * nr; e += 64) {
      const int r = e / cnt, j = e - r * cnt;
      xr[wv][j][r] = x[r * rh.ldx + R[jc + j]];
    }
    wave_lds_sync();
    if (i < ns) {
      double u[JC];
#pragma unroll
      for (int j = 0; j < JC; ++j) u[j] = j < cnt ? U12[(jc + j) * ns + i] : 0.0;
#pragma unroll
      for (int j = 0; j < JC; ++j) {
        if (j < cnt) {
#pragma unroll
          for (int r = 0; r < NR; ++r)
            if (r < nr) acc[r] = fma(u[j], xr[wv][j][r], acc[r]);
        }
      }
    }
    wave_lds_sync();   // every lane's reads of this chunk before the next chunk overwrites it
  }
#pragma unroll
  for (int r = 0; r < NR; ++r)
    if (r < nr) part[wv][r][lane] = acc[r];
  __syncthreads();
  if (wv == 0 && i < ns)
    for (int r = 0; r < nr; ++r) {
      double t = part[0][r][lane];
#pragma unroll
      for (int w = 1; w < W; ++w) t += part[w][r][lane];
      vbuf[r * rh.ldv + s.voff + i] = x[r * rh.ldx + s.first + i] - t;
    }
}

// ------------------------------------------------------------------------------------
// Multi-GPU helpers.  k_segcopy: the pack / unpack copies of an exchange, one workgroup per
// segment (4-byte words).  k_bwd_u12_cols: backward-solve contribution of one update-column
// block of a shared front, v[i] (-)= sum_{j in [c0, c1)} U[i, j] x[R[j - ns]] for i < ns
// (U12 rows of the block at U + (j - c0) * ns); init: v[i] = x[first + i] - sum.
// k_vcopy: v[i] = x[first + i], i < ns (start of the backward chain of a front without U12).
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_segcopy(const SegDesc* __restrict__ d, int64_t nd) {
  for (int64_t k = blockIdx.x; k < nd; k += gridDim.x) {
    const SegDesc g = d[k];
    const uint32_t* s = reinterpret_cast<const uint32_t*>(g.src);
    uint32_t* t = reinterpret_cast<uint32_t*>(g.dst);
    for (int64_t i = threadIdx.x; i < g.n4; i += 256) t[i] = s[i];
  }
}
__global__ __launch_bounds__(256) void k_bwd_u12_cols(const SNode* __restrict__ sn, int node, int64_t c0,
                                                      int64_t c1, int init, const int32_t* __restrict__ rows,
                                                      const double* __restrict__ store,
                                                      const double* __restrict__ x, double* __restrict__ vbuf) {
  const SNode s = sn[node];
  const int64_t ns = s.ns;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= ns) return;
  const int32_t* R = rows + s.rowptr;
  const double* U = store + s.Uoff;
  double acc = 0.0;
  for (int64_t j = c0; j < c1; ++j) acc = fma(U[(j - ns) * ns + i], x[R[j - ns]], acc);
  double* v = vbuf + s.voff;
  v[i] = (init ? x[s.first + i] : v[i]) - acc;
}
__global__ void k_vcopy(const SNode* __restrict__ sn, int node, const double* __restrict__ x,
                        double* __restrict__ vbuf) {
  const SNode s = sn[node];
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < s.ns) vbuf[s.voff + i] = x[s.first + i];
}

// wrk[r][i] = Rs[p0[i]] * b[r][p0[i]]   (blockIdx.y = right-hand side)
__global__ void k_perm_in(int64_t n, const int64_t* __restrict__ p0, const double* __restrict__ Rs,
                          const double* __restrict__ b, int64_t ldb, double* __restrict__ wrk, int64_t ldw) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    int64_t r = p0[i];
    wrk[blockIdx.y * ldw + i] = Rs[r] * b[blockIdx.y * ldb + r];
  }
}
// x[r][q[i]] = wrk[r][i]
__global__ void k_perm_out(int64_t n, const int64_t* __restrict__ q, const double* __restrict__ wrk, int64_t ldw,
                           double* __restrict__ x, int64_t ldx) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[blockIdx.y * ldx + q[i]] = wrk[blockIdx.y * ldw + i];
}
// final order -> pre-swap positions: out[first + rowperm[first+i]] = in[first+i]
__global__ void k_unswap(int64_t n, const int64_t* __restrict__ pos_first,
                         const int32_t* __restrict__ rowperm, const double* __restrict__ in,
                         double* __restrict__ out) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    int64_t f = pos_first[i];
    out[f + rowperm[i]] = in[i];
  }
}



// ------------------------------------------------------------------------------------
// Iterative refinement (pivot-failure fallback): r = b - A x by rows of A (entries of a row in
// column order, deterministic), max |r_i| into nrm[0] and the componentwise backward error
// max_i |r_i| / (|A| |x| + |b|)_i (Oettli-Prager; LAPACK dgerfs' BERR, a row with a zero
// denominator and r_i = 0 counts 0) into nrm[1]; x += d.
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_residual(int64_t n, const int64_t* __restrict__ rowptr,
                                                  const int32_t* __restrict__ ent,
                                                  const int32_t* __restrict__ acol,
                                                  const double* __restrict__ a,
                                                  const double* __restrict__ x,
                                                  const double* __restrict__ b, double* __restrict__ r,
                                                  double* __restrict__ nrm) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  double ri = 0.0, wi = 0.0;
  if (i < n) {
    double acc = 0.0, den = 0.0;
    for (int64_t e = rowptr[i]; e < rowptr[i + 1]; ++e) {
      const int32_t k = ent[e];
      const double xk = x[acol[k]];
      acc = fma(a[k], xk, acc);
      den = fma(fabs(a[k]), fabs(xk), den);
    }
    ri = b[i] - acc;
    r[i] = ri;
    den += fabs(b[i]);
    wi = ri == 0.0 ? 0.0 : den > 0.0 ? fabs(ri) / den : HUGE_VAL;
  }
  const double m = wave_max(fabs(ri));
  const double w = wave_max(wi);
  if ((threadIdx.x & 63) == 0 && m > 0.0) atomic_max_pos(nrm, m);
  if ((threadIdx.x & 63) == 0 && w > 0.0) atomic_max_pos(nrm + 1, w);
}
// Diagonal dominance of A's current values in HBM (the device twin of smlu.cpp's host
// diagonally_dominant(), for smlu_refactor_device): thread i sums |column i| in CSC order and
// |row i| over its entries in column order (Arow_ent), the host's summation order, so both take
// the same decision; flags[0] / flags[1] are cleared when some column / row is not dominant.
__global__ void k_dom_init(int32_t* __restrict__ flags) {
  if (threadIdx.x < 2) flags[threadIdx.x] = 1;
}
__global__ __launch_bounds__(256) void k_dominance(int64_t n, const int64_t* __restrict__ colptr,
                                                   const int32_t* __restrict__ arow,
                                                   const int64_t* __restrict__ rowptr,
                                                   const int32_t* __restrict__ ent,
                                                   const int32_t* __restrict__ acol,
                                                   const double* __restrict__ a, int32_t* __restrict__ flags) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  // entries eight at a time (all loads of a group in flight together), summed in order
  double d = 0.0, off = 0.0;
  const int64_t c1 = colptr[i + 1];
  for (int64_t e0 = colptr[i]; e0 < c1; e0 += 8) {
    double v[8];
    int32_t r[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      v[k] = e0 + k < c1 ? a[e0 + k] : 0.0;
      r[k] = e0 + k < c1 ? arow[e0 + k] : -1;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (r[k] < 0) continue;
      if (r[k] == i) d += fabs(v[k]);
      else off += fabs(v[k]);
    }
  }
  if (!(d > 0.0 && d >= off)) flags[0] = 0;
  d = 0.0;
  off = 0.0;
  const int64_t r1 = rowptr[i + 1];
  for (int64_t t0 = rowptr[i]; t0 < r1; t0 += 8) {
    int32_t e[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) e[k] = t0 + k < r1 ? ent[t0 + k] : -1;
    double v[8];
    int32_t c[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      v[k] = e[k] >= 0 ? a[e[k]] : 0.0;
      c[k] = e[k] >= 0 ? acol[e[k]] : -1;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (e[k] < 0) continue;
      if (c[k] == i) d += fabs(v[k]);
      else off += fabs(v[k]);
    }
  }
  if (!(d > 0.0 && d >= off)) flags[1] = 0;
}
// Status record of a factorization / dominance test / solve for the host (smlu.cpp: read_status):
// out[0] = out[15] = seq (the host accepts a copy only when both match its own sequence number);
// with info: out[1] = weak-pivot nodes, out[2], out[3] = first zero-pivot node and its info word
// (-1, 0: none), out[4], out[5] = first flagged node and its word; out[6] = words[0] | words[1] << 32,
// out[7] = words[2] | words[3] << 32 (up to 4 status words);
// out[8], out[9] = first node whose info word is outside the legal code set and that word (-1, 0:
// none), out[10] = how many such nodes.  Legal words are the ones publish_info / the growth epilogues
// write: bit 0 zero pivot, bit 1 weak pivot, bits 2.. = 1 + the front-local column of the first zero
// pivot, at most ns (0 <= v < (ns + 1) << 2).  Any other word is not a pivot status and is never
// read as one (the host fails with SMLU_ERR_STATE).  One workgroup of 1024 threads; above
// kStatusSplit nodes the scan runs first over kStatusParts workgroups (k_status_part, five partial
// results each at out[16 + 5 p ...]) and k_status reduces those (128^3: 0.54 ms -> a few us).
constexpr int64_t kStatusSplit = 16384;
constexpr int kStatusParts = 512;
struct StatusAcc {
  long long weak = 0, nbad = 0, sing = LLONG_MAX, flag = LLONG_MAX, bad = LLONG_MAX;
};
__device__ __forceinline__ void status_scan(StatusAcc& a, const int32_t* __restrict__ info, const SNode* __restrict__ sn,
                                            int64_t i0, int64_t nnodes, int64_t stride) {
  for (int64_t i = i0; i < nnodes; i += stride) {
    const int32_t v = info[i];
    const bool legal = v >= 0 && (!sn || (int64_t)v < (((int64_t)sn[i].ns + 1) << 2));
    if (!legal) {
      ++a.nbad;
      if (i < a.bad) a.bad = i;
      continue;
    }
    a.weak += (v >> 1) & 1;
    if ((v & 1) && i < a.sing) a.sing = i;
    if ((v & 3) && i < a.flag) a.flag = i;
  }
}
// workgroup reduction of the five fields (NT threads), result in s_*[0]
template <int NT>
__device__ __forceinline__ void status_reduce(StatusAcc a, long long* s_weak, long long* s_nbad, long long* s_sing,
                                              long long* s_flag, long long* s_bad) {
  const int tid = threadIdx.x;
  s_weak[tid] = a.weak;
  s_nbad[tid] = a.nbad;
  s_sing[tid] = a.sing;
  s_flag[tid] = a.flag;
  s_bad[tid] = a.bad;
  __syncthreads();
  for (int w = NT / 2; w > 0; w >>= 1) {
    if (tid < w) {
      s_weak[tid] += s_weak[tid + w];
      s_nbad[tid] += s_nbad[tid + w];
      s_sing[tid] = min(s_sing[tid], s_sing[tid + w]);
      s_flag[tid] = min(s_flag[tid], s_flag[tid + w]);
      s_bad[tid] = min(s_bad[tid], s_bad[tid + w]);
    }
    __syncthreads();
  }
}
__global__ __launch_bounds__(256) void k_status_part(const int32_t* __restrict__ info, int64_t nnodes,
                                                     const SNode* __restrict__ sn, long long* __restrict__ part) {
  __shared__ long long s_weak[256], s_nbad[256], s_sing[256], s_flag[256], s_bad[256];
  StatusAcc a;
  status_scan(a, info, sn, (int64_t)blockIdx.x * 256 + threadIdx.x, nnodes, (int64_t)gridDim.x * 256);
  status_reduce<256>(a, s_weak, s_nbad, s_sing, s_flag, s_bad);
  if (threadIdx.x == 0) {
    long long* o = part + 5 * blockIdx.x;
    o[0] = s_weak[0];
    o[1] = s_nbad[0];
    o[2] = s_sing[0];
    o[3] = s_flag[0];
    o[4] = s_bad[0];
  }
}
__global__ __launch_bounds__(1024) void k_status(const int32_t* __restrict__ info, int64_t nnodes,
                                                 const SNode* __restrict__ sn,
                                                 const int32_t* __restrict__ words, int nwords,
                                                 long long* __restrict__ out, long long seq, int nparts) {
  __shared__ long long s_weak[1024], s_nbad[1024];
  __shared__ long long s_sing[1024], s_flag[1024], s_bad[1024];
  const int tid = threadIdx.x;
  StatusAcc a;
  if (info && nparts > 0) {
    if (tid < nparts) {
      const long long* o = out + 16 + 5 * tid;
      a.weak = o[0];
      a.nbad = o[1];
      a.sing = o[2];
      a.flag = o[3];
      a.bad = o[4];
    }
  } else if (info) {
    status_scan(a, info, sn, tid, nnodes, 1024);
  }
  status_reduce<1024>(a, s_weak, s_nbad, s_sing, s_flag, s_bad);
  if (tid == 0) {
    const long long sg = s_sing[0], fl = s_flag[0], bd = s_bad[0];
    out[1] = s_weak[0];
    out[2] = sg == LLONG_MAX ? -1 : sg;
    out[3] = sg == LLONG_MAX ? 0 : info[sg];
    out[4] = fl == LLONG_MAX ? -1 : fl;
    out[5] = fl == LLONG_MAX ? 0 : info[fl];
    const long long w0 = nwords > 0 ? (long long)(uint32_t)words[0] : 0;
    const long long w1 = nwords > 1 ? (long long)(uint32_t)words[1] : 0;
    const long long w2 = nwords > 2 ? (long long)(uint32_t)words[2] : 0;
    const long long w3 = nwords > 3 ? (long long)(uint32_t)words[3] : 0;
    out[6] = w0 | (w1 << 32);
    out[7] = w2 | (w3 << 32);
    out[8] = bd == LLONG_MAX ? -1 : bd;
    out[9] = bd == LLONG_MAX ? 0 : info[bd];
    out[10] = s_nbad[0];
    for (int i = 11; i < 15; ++i) out[i] = 0;
    out[0] = seq;
    out[15] = seq;
  }
}
// Dev (tools/determinism.py): an order-independent 64-bit hash per front of its factor values
// (L panel + U12, bit patterns) and of its row permutation, to localise a factorization that
// differs between two runs on the same values.  One workgroup per front.
__device__ __forceinline__ unsigned long long mix64(unsigned long long x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  return x ^ (x >> 33);
}
__global__ __launch_bounds__(256) void k_front_hash(const SNode* __restrict__ sn, const double* __restrict__ store,
                                                    const int32_t* __restrict__ rowperm,
                                                    unsigned long long* __restrict__ out) {
  __shared__ unsigned long long hv, hp;
  const SNode r = sn[blockIdx.x];
  const int64_t M = (int64_t)r.ns + r.nu;
  if (threadIdx.x == 0) hv = hp = 0;
  __syncthreads();
  unsigned long long a = 0, b = 0;
  const int64_t nl = M * r.ns, nu12 = (int64_t)r.ns * r.nu;
  for (int64_t i = threadIdx.x; i < nl + nu12; i += 256) {
    const double v = i < nl ? store[r.Loff + i] : store[r.Uoff + (i - nl)];
    a += mix64((unsigned long long)__double_as_longlong(v) + 0x9e3779b97f4a7c15ull * (unsigned long long)(i + 1));
  }
  for (int64_t i = threadIdx.x; i < r.ns; i += 256)
    b += mix64((unsigned long long)(uint32_t)rowperm[r.first + i] * 0x9e3779b97f4a7c15ull + (unsigned long long)i);
  atomicAdd(&hv, a);
  atomicAdd(&hp, b);
  __syncthreads();
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = hv;
    out[2 * blockIdx.x + 1] = hp;
  }
}
__global__ void k_axpy1(int64_t n, const double* __restrict__ d, double* __restrict__ x) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[i] += d[i];
}
// ComplexF64 values (interleaved re, im per entry of A's CSC) -> the real-equivalent K's values:
// entry e of complex column j lands as (re, im) at dst[e] (column 2j) and as (-im, re) at
// dst[e] + off[e] (column 2j+1).  One lane per complex entry, 16-byte loads, two 16-byte stores.
__global__ void k_expand_z(int64_t nnz, const double2* __restrict__ z, const int64_t* __restrict__ dst,
                           const int32_t* __restrict__ off, double* __restrict__ K) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= nnz) return;
  const double2 v = z[e];
  const int64_t d = dst[e];
  *reinterpret_cast<double2*>(K + d) = v;
  *reinterpret_cast<double2*>(K + d + off[e]) = make_double2(-v.y, v.x);
}

// ------------------------------------------------------------------------------------
// Host-side launch wrappers (called from smlu.cpp)
// ------------------------------------------------------------------------------------
static inline unsigned nblk(int64_t n, int b) { return (unsigned)((n + b - 1) / b); }
hipError_t launch_fwd(hipStream_t st, int cnt, const int32_t* list, const SNode* sn,
                      const int32_t* chlist, const int32_t* relmap, const int32_t* rowperm,
                      const double* store, double* x, double* vbuf, Rhs rh) {
  if (cnt <= 0) return hipSuccess;
  if (rh.n < 1 || rh.n > kMaxRhs) return hipErrorInvalidValue;
  if (rh.n == 1) k_fwd_front<1><<<cnt, 256, 0, st>>>(list, sn, chlist, relmap, rowperm, store, x, vbuf, rh);
  else if (rh.n <= 4) k_fwd_front<4><<<cnt, 256, 0, st>>>(list, sn, chlist, relmap, rowperm, store, x, vbuf, rh);
  else if (rh.n <= 8) k_fwd_front<8><<<cnt, 256, 0, st>>>(list, sn, chlist, relmap, rowperm, store, x, vbuf, rh);
  else k_fwd_front<16><<<cnt, 256, 0, st>>>(list, sn, chlist, relmap, rowperm, store, x, vbuf, rh);
  return hipGetLastError();
}
hipError_t launch_bwd(hipStream_t st, int cnt, const int32_t* list, const SNode* sn,
                      const int32_t* rows, const double* store, double* x, double* vbuf, Rhs rh) {
  if (cnt <= 0) return hipSuccess;
  if (rh.n < 1 || rh.n > kMaxRhs) return hipErrorInvalidValue;
  if (rh.n == 1) k_bwd_front<1><<<cnt, 256, 0, st>>>(list, sn, rows, store, x, vbuf, rh);
  else if (rh.n <= 4) k_bwd_front<4><<<cnt, 256, 0, st>>>(list, sn, rows, store, x, vbuf, rh);
  else if (rh.n <= 8) k_bwd_front<8><<<cnt, 256, 0, st>>>(list, sn, rows, store, x, vbuf, rh);
  else k_bwd_front<16><<<cnt, 256, 0, st>>>(list, sn, rows, store, x, vbuf, rh);
  return hipGetLastError();
}
hipError_t launch_fwd_tiny(hipStream_t st, int cnt, const int32_t* list, const SNode* sn,
                           const int32_t* chlist, const int32_t* relmap, const int32_t* rowperm,
                           const double* store, double* x, double* vbuf, Rhs rh, int micro) {
  if (cnt <= 0) return hipSuccess;
  if (rh.n < 1 || rh.n > kMaxRhs) return hipErrorInvalidValue;
  if (micro) {   // every front of the list has M <= 8 (batches too: the rows loaded once per front)
    k_fwd_micro<<<nblk(cnt, 32), 256, 0, st>>>(list, cnt, sn, chlist, relmap, rowperm, store, x, vbuf, rh);
    return hipGetLastError();
  }
  const unsigned g = nblk(cnt, 4);
  if (rh.n == 1) k_fwd_tiny<1><<<g, 256, 0, st>>>(list, cnt, sn, chlist, relmap, rowperm, store, x, vbuf, rh);
  else if (rh.n <= 8) k_fwd_tiny<8><<<g, 256, 0, st>>>(list, cnt, sn, chlist, relmap, rowperm, store, x, vbuf, rh);
  else k_fwd_tiny<kMaxRhs><<<g, 256, 0, st>>>(list, cnt, sn, chlist, relmap, rowperm, store, x, vbuf, rh);
  return hipGetLastError();
}
hipError_t launch_bwd_tiny(hipStream_t st, int cnt, const int32_t* list, const SNode* sn,
                           const int32_t* rows, const double* store, double* x, double* vbuf, Rhs rh, int micro) {
  if (cnt <= 0) return hipSuccess;
  if (rh.n < 1 || rh.n > kMaxRhs) return hipErrorInvalidValue;
  if (micro) {
    k_bwd_micro<<<nblk(cnt, 32), 256, 0, st>>>(list, cnt, sn, rows, store, x, vbuf, rh);
    return hipGetLastError();
  }
  const unsigned g = nblk(cnt, 4);
  // the <4> instance also for a single rhs: <1> lets the compiler keep the U12 and U11 slabs live
  // together (256 VGPRs)
  if (rh.n <= 4) k_bwd_tiny<4><<<g, 256, 0, st>>>(list, cnt, sn, rows, store, x, vbuf, rh);
  else if (rh.n <= 8) k_bwd_tiny<8><<<g, 256, 0, st>>>(list, cnt, sn, rows, store, x, vbuf, rh);
  else k_bwd_tiny<kMaxRhs><<<g, 256, 0, st>>>(list, cnt, sn, rows, store, x, vbuf, rh);
  return hipGetLastError();
}
hipError_t launch_fwd_pull(hipStream_t st, int64_t nwg, const FrontTile* ft, int nft, const SNode* sn,
                           const int32_t* rowperm, const int32_t* gptr, const int32_t* gent, const double* x,
                           double* vbuf, Rhs rh) {
  if (nwg <= 0) return hipSuccess;
#define PULL(NR) k_fwd_pull<NR><<<(unsigned)nwg, 256, 0, st>>>(ft, nft, sn, rowperm, gptr, gent, x, vbuf, rh)
  if (rh.n <= 1) PULL(1);
  else if (rh.n <= 4) PULL(4);
  else if (rh.n <= 8) PULL(8);
  else PULL(16);
#undef PULL
  return hipGetLastError();
}
hipError_t launch_fwd_gather(hipStream_t st, int cnt, const int32_t* list, const SNode* sn,
                             const int32_t* chlist, const int32_t* relmap, const int32_t* rowperm,
                             double* x, double* vbuf, Rhs rh) {
  if (cnt <= 0) return hipSuccess;
  if (rh.n < 1 || rh.n > kMaxRhs) return hipErrorInvalidValue;
  k_fwd_gather<<<dim3((unsigned)cnt, (unsigned)rh.n), 256, 0, st>>>(list, sn, chlist, relmap, rowperm, x, vbuf, rh);
  return hipGetLastError();
}
hipError_t launch_tri_block(hipStream_t st, bool upper, int64_t nwg, const FrontTile* ft, int nft,
                            int step, const SNode* sn, const double* store, double* x, double* vbuf, Rhs rh) {
  if (nwg <= 0) return hipSuccess;
  if (rh.n < 1 || rh.n > kMaxRhs) return hipErrorInvalidValue;
  // one chain wave for a single vector (320 threads), four for a batch (512)
#define SMLU_TRI(NRV, THR)                                                                           \
  (upper ? (k_tri_block<true, NRV><<<(unsigned)nwg, THR, 0, st>>>(ft, nft, step, sn, store, x, vbuf, rh)) \
         : (k_tri_block<false, NRV><<<(unsigned)nwg, THR, 0, st>>>(ft, nft, step, sn, store, x, vbuf, rh)))
  if (rh.n == 1) SMLU_TRI(1, 320);
  else if (rh.n <= 4) SMLU_TRI(4, 512);
  else if (rh.n <= 8) SMLU_TRI(8, 512);
  else SMLU_TRI(16, 512);
#undef SMLU_TRI
  return hipGetLastError();
}
hipError_t launch_bwd_u12(hipStream_t st, int64_t nwg, const FrontTile* ft, int nft, const SNode* sn,
                          const int32_t* rows, const double* store, const double* x, double* vbuf, Rhs rh) {
  if (nwg <= 0) return hipSuccess;
  if (rh.n < 1 || rh.n > kMaxRhs) return hipErrorInvalidValue;
  // accumulators per right-hand side in registers: instantiate for the batch width
  if (rh.n == 1) k_bwd_u12<1><<<(unsigned)nwg, 512, 0, st>>>(ft, nft, sn, rows, store, x, vbuf, rh);
  else if (rh.n <= 4) k_bwd_u12<4><<<(unsigned)nwg, 512, 0, st>>>(ft, nft, sn, rows, store, x, vbuf, rh);
  else if (rh.n <= 8) k_bwd_u12<8><<<(unsigned)nwg, 512, 0, st>>>(ft, nft, sn, rows, store, x, vbuf, rh);
  else k_bwd_u12<16><<<(unsigned)nwg, 512, 0, st>>>(ft, nft, sn, rows, store, x, vbuf, rh);
  return hipGetLastError();
}
hipError_t launch_tri_sweep(hipStream_t st, bool upper, int64_t nwg, const FrontTile* ft, int nft,
                            unsigned long long* tick, int32_t* flags, double* xh, int32_t* status, const SNode* sn,
                            const double* store, double* x, double* vbuf, Rhs rh, int spin) {
  if (nwg <= 0) return hipSuccess;
  // up to 8 right-hand sides (NR-wide hand-off slots); wider batches take the per-block schedule
  if (rh.n < 1 || rh.n > 8) return hipErrorInvalidValue;
#define SWEEP(NR)                                                                                                   \
  (upper ? (k_tri_sweep<true, NR><<<(unsigned)nwg, 64 * kSweepWK, 0, st>>>(ft, nft, tick, flags, xh, status, sn, store, x, vbuf, rh, spin)) \
         : (k_tri_sweep<false, NR><<<(unsigned)nwg, 64 * kSweepWK, 0, st>>>(ft, nft, tick, flags, xh, status, sn, store, x, vbuf, rh, spin)))
  if (rh.n == 1) SWEEP(1);
  else if (rh.n <= 4) SWEEP(4);
  else SWEEP(8);
#undef SWEEP
  return hipGetLastError();
}
hipError_t launch_residual(hipStream_t st, int64_t n, const int64_t* rowptr, const int32_t* ent,
                           const int32_t* acol, const double* a, const double* x, const double* b,
                           double* r, double* nrm) {
  if (n <= 0) return hipSuccess;
  k_residual<<<nblk(n, 256), 256, 0, st>>>(n, rowptr, ent, acol, a, x, b, r, nrm);
  return hipGetLastError();
}
hipError_t launch_dominance(hipStream_t st, int64_t n, const int64_t* colptr, const int32_t* arow,
                            const int64_t* rowptr, const int32_t* ent, const int32_t* acol, const double* a,
                            int32_t* dflags) {
  k_dom_init<<<1, 64, 0, st>>>(dflags);   // (a kernel: no pageable host-to-device copy)
  if (n > 0) k_dominance<<<nblk(n, 256), 256, 0, st>>>(n, colptr, arow, rowptr, ent, acol, a, dflags);
  return hipGetLastError();
}
hipError_t launch_front_hash(hipStream_t st, int64_t nsup, const SNode* sn, const double* store, const int32_t* rowperm,
                             unsigned long long* out) {
  if (nsup <= 0) return hipSuccess;
  k_front_hash<<<(unsigned)nsup, 256, 0, st>>>(sn, store, rowperm, out);
  return hipGetLastError();
}
hipError_t launch_status(hipStream_t st, const int32_t* info, int64_t nnodes, const SNode* sn, const int32_t* words,
                         int nwords, long long* out, long long seq) {
  int nparts = 0;
  if (info && nnodes > kStatusSplit) {   // out holds 16 + 5 * kStatusParts words (schedule.cpp)
    nparts = kStatusParts;
    k_status_part<<<(unsigned)nparts, 256, 0, st>>>(info, nnodes, sn, out + 16);
  }
  k_status<<<1, 1024, 0, st>>>(info, nnodes, sn, words, nwords, out, seq, nparts);
  return hipGetLastError();
}
hipError_t launch_axpy1(hipStream_t st, int64_t n, const double* d, double* x) {
  if (n <= 0) return hipSuccess;
  k_axpy1<<<nblk(n, 256), 256, 0, st>>>(n, d, x);
  return hipGetLastError();
}
hipError_t launch_expand_z(hipStream_t st, int64_t nnz, const double* z, const int64_t* dst, const int32_t* off,
                           double* K) {
  if (nnz <= 0) return hipSuccess;
  k_expand_z<<<nblk(nnz, 256), 256, 0, st>>>(nnz, reinterpret_cast<const double2*>(z), dst, off, K);
  return hipGetLastError();
}
hipError_t launch_perm_in(hipStream_t st, int64_t n, const int64_t* p0, const double* Rs,
                          const double* b, double* wrk, int nrhs, int64_t ldb, int64_t ldw) {
  k_perm_in<<<dim3(nblk(n, 256), (unsigned)nrhs), 256, 0, st>>>(n, p0, Rs, b, ldb, wrk, ldw);
  return hipGetLastError();
}
hipError_t launch_segcopy(hipStream_t st, const SegDesc* d, int64_t nd) {
  if (nd <= 0) return hipSuccess;
  k_segcopy<<<(unsigned)std::min<int64_t>(nd, 65535), 256, 0, st>>>(d, nd);
  return hipGetLastError();
}
hipError_t launch_bwd_u12_cols(hipStream_t st, const SNode* sn, int node, int64_t ns, int64_t c0, int64_t c1,
                               int init, const int32_t* rows, const double* store, const double* x,
                               double* vbuf) {
  if (ns <= 0) return hipSuccess;
  k_bwd_u12_cols<<<nblk(ns, 256), 256, 0, st>>>(sn, node, c0, c1, init, rows, store, x, vbuf);
  return hipGetLastError();
}
hipError_t launch_vcopy(hipStream_t st, const SNode* sn, int node, int64_t ns, const double* x, double* vbuf) {
  if (ns <= 0) return hipSuccess;
  k_vcopy<<<nblk(ns, 256), 256, 0, st>>>(sn, node, x, vbuf);
  return hipGetLastError();
}
// ------------------------------------------------------------------------------------
// The reference's chunked triangular solves: lsolve! (src/SharedMemSparseLU.jl:
// 349-367) and rsolve! (:374-392) chunk by chunk in the reference's order -- trsv! on the
// diagonal block (dtrsv 'L','N','U' / 'U','N','N', column sweep), then x[rows] += Rect*x[cols]
// with the negated rectangle (gemm! with alpha = beta = 1, quirk Q3).  One workgroup walks the
// chunks in sequence (each chunk depends on the previous); rectangle rows are spread over its
// 256 threads.  A parity mode for small banded systems, not the fast path.
// ------------------------------------------------------------------------------------
template <bool UPPER>
__global__ __launch_bounds__(256) void k_chunked_solve(int64_t nchunk, const ChunkDesc* __restrict__ desc,
                                                       const double* __restrict__ data,
                                                       double* __restrict__ x) {
  for (int64_t c = 0; c < nchunk; ++c) {
    const ChunkDesc d = desc[c];
    const double* T = data + d.tri;
    double* xs = x + d.c0;
    if (threadIdx.x == 0) {
      if (!UPPER) {
        for (int64_t j = 0; j < d.s; ++j) {
          const double xj = xs[j];
          for (int64_t i = j + 1; i < d.s; ++i) xs[i] = fma(-T[j * d.s + i], xj, xs[i]);
        }
      } else {
        for (int64_t j = d.s - 1; j >= 0; --j) {
          xs[j] = xs[j] / T[j * d.s + j];
          const double xj = xs[j];
          for (int64_t i = 0; i < j; ++i) xs[i] = fma(-T[j * d.s + i], xj, xs[i]);
        }
      }
    }
    __syncthreads();
    const double* Rc = data + d.rect;
    for (int64_t r = threadIdx.x; r < d.nr; r += 256) {
      double acc = x[d.r0 + r];
      for (int64_t j = 0; j < d.s; ++j) acc = fma(Rc[j * d.nr + r], xs[j], acc);
      x[d.r0 + r] = acc;
    }
    __syncthreads();
  }
}

hipError_t launch_chunked_solve(hipStream_t st, bool upper, int64_t nchunk, const ChunkDesc* desc,
                                const double* data, double* x) {
  if (nchunk <= 0) return hipSuccess;
  if (upper) k_chunked_solve<true><<<1, 256, 0, st>>>(nchunk, desc, data, x);
  else k_chunked_solve<false><<<1, 256, 0, st>>>(nchunk, desc, data, x);
  return hipGetLastError();
}

hipError_t launch_perm_out(hipStream_t st, int64_t n, const int64_t* q, const double* wrk, double* x, int nrhs,
                           int64_t ldw, int64_t ldx) {
  k_perm_out<<<dim3(nblk(n, 256), (unsigned)nrhs), 256, 0, st>>>(n, q, wrk, ldw, x, ldx);
  return hipGetLastError();
}
hipError_t launch_unswap(hipStream_t st, int64_t n, const int64_t* pos_first, const int32_t* rowperm,
                         const double* in, double* out) {
  k_unswap<<<nblk(n, 256), 256, 0, st>>>(n, pos_first, rowperm, in, out);
  return hipGetLastError();
}


}  // namespace smlu


#ifdef SMLU_SWEEP_TRACE
// Dev hook for tools/sweep_trace.py: nwg > 0 arms the trace for sweeps of that grid and direction
// (n records of 8 clocks); nwg == 0 copies the records to out and disarms.
extern "C" int smlu_dev_sweep_trace(int nwg, int upper, long long* out, long long n) {
  static long long* buf = nullptr;
  using namespace smlu;
  SweepTrace t{nullptr, 0, 0};
  if (nwg > 0) {
    if (buf) (void)hipFree(buf);
    if (hipMalloc(&buf, sizeof(long long) * 8 * n) != hipSuccess) return -1;
    (void)hipMemset(buf, 0, sizeof(long long) * 8 * n);
    t = SweepTrace{buf, nwg, upper};
  } else if (buf) {
    (void)hipDeviceSynchronize();
    if (out && hipMemcpy(out, buf, sizeof(long long) * 8 * n, hipMemcpyDeviceToHost) != hipSuccess) return -1;
  }
  return hipMemcpyToSymbol(HIP_SYMBOL(g_sweep_trace), &t, sizeof t) == hipSuccess ? 0 : -1;
}
#endif
