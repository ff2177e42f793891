// kernels_solve.hip — level-scheduled forward/backward solves (lsolve!/rsolve!, src/SharedMemSparseLU.jl:349-392)
// and ldiv!'s scale/permute steps (:318-339).
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
template <bool UPPER>
__device__ __forceinline__ double tri_lds(double xi, const double* __restrict__ sD, int bw, int lane) {
  if (!UPPER) {
    for (int j = 0; j < bw; ++j) {
      const double xj = readlane_f64(xi, j);
      if (lane > j && lane < bw) xi = fma(-sD[j * 65 + lane], xj, xi);
    }
  } else {
    for (int j = bw - 1; j >= 0; --j) {
      if (lane == j) xi = xi * recip(sD[j * 65 + j]);
      const double xj = readlane_f64(xi, j);
      if (lane < j) xi = fma(-sD[j * 65 + lane], xj, xi);
    }
  }
  return xi;
}

__global__ __launch_bounds__(256) void k_fwd_front(const int32_t* __restrict__ list,
                                                   const SNode* __restrict__ sn,
                                                   const int32_t* __restrict__ chlist,
                                                   const int32_t* __restrict__ relmap,
                                                   const int32_t* __restrict__ rowperm,
                                                   const double* __restrict__ store,
                                                   double* __restrict__ x,
                                                   double* __restrict__ vbuf) {
  __shared__ double xs[64];
  __shared__ double sD[64 * 65];
  const SNode s = sn[list[blockIdx.x]];
  const int64_t M = (int64_t)s.ns + s.nu, ns = s.ns;
  double* v = vbuf + s.voff;
  double* xo = x + s.first;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  for (int64_t i = tid; i < M; i += 256) v[i] = i < ns ? xo[i] : 0.0;
  __syncthreads();
  for (int c = s.chbeg; c < s.chend; ++c) {
    const SNode ch = sn[chlist[c]];
    const double* u = vbuf + ch.voff + ch.ns;
    const int32_t* rm = relmap + ch.rowptr;
    for (int64_t i = tid; i < ch.nu; i += 256) v[rm[i]] += u[i];
    __syncthreads();
  }
  // permuted diagonal-block right-hand side -> x positions (owned by this front)
  for (int64_t i = tid; i < ns; i += 256) xo[i] = v[rowperm[s.first + i]];
  __syncthreads();
  for (int64_t i = tid; i < ns; i += 256) v[i] = xo[i];
  __syncthreads();
  const double* Lp = store + s.Loff;
  for (int64_t jb = 0; jb < ns; jb += 64) {
    const int bw = (int)min<int64_t>(64, ns - jb);
    stage_block(sD, Lp + jb * M + jb, M, bw, tid);
    __syncthreads();
    if (wv == 0) {
      double xi = lane < bw ? v[jb + lane] : 0.0;
      xi = tri_lds<false>(xi, sD, bw, lane);
      if (lane < bw) {
        xs[lane] = xi;
        v[jb + lane] = xi;
      }
    }
    __syncthreads();
    for (int64_t i = jb + bw + tid; i < M; i += 256) {
      double acc = 0.0;
#pragma unroll 8
      for (int j = 0; j < bw; ++j) acc = fma(Lp[(jb + j) * M + i], xs[j], acc);
      v[i] -= acc;
    }
    __syncthreads();
  }
  for (int64_t i = tid; i < ns; i += 256) xo[i] = v[i];
}

// Backward (U): x_s -= U12 * x[R_s]; then upper solve of the diagonal block from the bottom.
__global__ __launch_bounds__(256) void k_bwd_front(const int32_t* __restrict__ list,
                                                   const SNode* __restrict__ sn,
                                                   const int32_t* __restrict__ rows,
                                                   const double* __restrict__ store,
                                                   double* __restrict__ x,
                                                   double* __restrict__ vbuf) {
  __shared__ double xs[64];
  __shared__ double sD[64 * 65];
  const SNode s = sn[list[blockIdx.x]];
  const int64_t M = (int64_t)s.ns + s.nu, ns = s.ns, nu = s.nu;
  double* v = vbuf + s.voff;
  double* xo = x + s.first;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int32_t* R = rows + s.rowptr;
  for (int64_t i = tid; i < nu; i += 256) v[ns + i] = x[R[i]];
  __syncthreads();
  const double* U12 = store + s.Uoff;
  for (int64_t i = tid; i < ns; i += 256) {
    double acc = 0.0;
#pragma unroll 8
    for (int64_t j = 0; j < nu; ++j) acc = fma(U12[j * ns + i], v[ns + j], acc);
    v[i] = xo[i] - acc;
  }
  __syncthreads();
  const double* Lp = store + s.Loff;  // U11 in the upper triangle of the L panel
  for (int64_t jb = ((ns - 1) / 64) * 64; jb >= 0; jb -= 64) {
    const int bw = (int)min<int64_t>(64, ns - jb);
    stage_block(sD, Lp + jb * M + jb, M, bw, tid);
    __syncthreads();
    if (wv == 0) {
      double xi = lane < bw ? v[jb + lane] : 0.0;
      xi = tri_lds<true>(xi, sD, bw, lane);
      if (lane < bw) {
        xs[lane] = xi;
        v[jb + lane] = xi;
      }
    }
    __syncthreads();
    for (int64_t i = tid; i < jb; i += 256) {
      double acc = 0.0;
#pragma unroll 8
      for (int j = 0; j < bw; ++j) acc = fma(Lp[(jb + j) * M + i], xs[j], acc);
      v[i] -= acc;
    }
    __syncthreads();
  }
  for (int64_t i = tid; i < ns; i += 256) xo[i] = v[i];
}

// ------------------------------------------------------------------------------------
// Solves for large fronts (ns > 256): the diagonal block sweep is split over workgroups.
// k_fwd_gather: front vector = own rows + children's update vectors, row permutation.
// k_fwd_block (step t, jb = 64t): every workgroup re-solves the 64x64 unit-lower diagonal
//   block from v (read-only in this launch), applies it to its 256-row chunk below; chunk 0
//   publishes the solved block into x.  k_bwd_u12: x_s -= U12 x[R_s] by row chunks.
// k_bwd_block: same as k_fwd_block for U11 from the bottom block up.
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_fwd_gather(const int32_t* __restrict__ list,
                                                    const SNode* __restrict__ sn,
                                                    const int32_t* __restrict__ chlist,
                                                    const int32_t* __restrict__ relmap,
                                                    const int32_t* __restrict__ rowperm,
                                                    double* __restrict__ x, double* __restrict__ vbuf) {
  const SNode s = sn[list[blockIdx.x]];
  const int64_t M = (int64_t)s.ns + s.nu, ns = s.ns;
  double* v = vbuf + s.voff;
  double* xo = x + s.first;
  const int tid = threadIdx.x;
  for (int64_t i = tid; i < M; i += 256) v[i] = i < ns ? xo[i] : 0.0;
  __syncthreads();
  for (int c = s.chbeg; c < s.chend; ++c) {
    const SNode ch = sn[chlist[c]];
    const double* u = vbuf + ch.voff + ch.ns;
    const int32_t* rm = relmap + ch.rowptr;
    for (int64_t i = tid; i < ch.nu; i += 256) v[rm[i]] += u[i];
    __syncthreads();
  }
  for (int64_t i = tid; i < ns; i += 256) xo[i] = v[rowperm[s.first + i]];
  __syncthreads();
  for (int64_t i = tid; i < ns; i += 256) v[i] = xo[i];
}

// One 64-column step of a large front: wave 0 of every workgroup solves the 64x64 diagonal
// block (tri64; each workgroup re-solves it, no inter-workgroup hand-off), waves 1-4 own one row
// each of the workgroup's 256-row chunk and load that row's 64 slab values before the solved
// block arrives (the two memory round trips overlap instead of following each other).
template <bool UPPER>
__global__ __launch_bounds__(320) void k_tri_block(const FrontTile* __restrict__ ft, int nft, int step,
                                                   const SNode* __restrict__ sn,
                                                   const double* __restrict__ store,
                                                   double* __restrict__ x, double* __restrict__ vbuf) {
  __shared__ double xs[64];
  const int64_t b = blockIdx.x;
  const int fi = find_front_tile(ft, nft, b);
  const SNode s = sn[ft[fi].s];
  const int64_t chunk = b - ft[fi].wg0;
  const int64_t M = (int64_t)s.ns + s.nu, ns = s.ns;
  const int64_t nblk = (ns + 63) / 64;
  const int64_t jb = UPPER ? (nblk - 1 - step) * 64 : (int64_t)step * 64;
  const int bw = (int)min<int64_t>(64, ns - jb);
  double* v = vbuf + s.voff;
  const double* Lp = store + s.Loff;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (wv == 0) {
    double xi = lane < bw ? v[jb + lane] : 0.0;
    xi = tri64<UPPER>(xi, Lp + jb * M + jb, M, bw, lane);
    if (lane < bw) {
      xs[lane] = xi;
      if (chunk == 0) x[s.first + jb + lane] = xi;
    }
    __syncthreads();
    return;
  }
  // rows updated by this chunk: forward -> [jb+bw, M), backward -> [0, jb)
  const int64_t r0 = UPPER ? chunk * 256 : jb + bw + chunk * 256;
  const int64_t r1 = UPPER ? jb : M;
  const int64_t i = r0 + tid - 64;
  const bool has = i < r1;
  double d[64];
#pragma unroll
  for (int j = 0; j < 64; ++j) d[j] = (has && j < bw) ? Lp[(jb + j) * M + i] : 0.0;
  __syncthreads();
  if (has) {
    double acc = 0.0;
#pragma unroll
    for (int j = 0; j < 64; ++j)
      if (j < bw) acc = fma(d[j], xs[j], acc);
    v[i] -= acc;
  }
}

// x_s[i] (in v) = x[first+i] - sum_j U12[i,j] * x[R_j], 256 rows per workgroup
// 64 rows per workgroup; wave w sums the columns [w*nu/4, (w+1)*nu/4) (x[R] staged in LDS
// per 64-column chunk, 8 loads in flight), the four partial sums combined in wave order.
__global__ __launch_bounds__(256) void k_bwd_u12(const FrontTile* __restrict__ ft, int nft,
                                                 const SNode* __restrict__ sn,
                                                 const int32_t* __restrict__ rows,
                                                 const double* __restrict__ store,
                                                 const double* __restrict__ x,
                                                 double* __restrict__ vbuf) {
  __shared__ double xr[4][64];
  __shared__ double part[4][64];
  const int64_t b = blockIdx.x;
  const int fi = find_front_tile(ft, nft, b);
  const SNode s = sn[ft[fi].s];
  const int64_t chunk = b - ft[fi].wg0;
  const int64_t ns = s.ns, nu = s.nu;
  const int32_t* R = rows + s.rowptr;
  const double* U12 = store + s.Uoff;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int64_t i = chunk * 64 + lane;
  const int64_t j0 = nu * wv / 4, j1 = nu * (wv + 1) / 4;
  double acc = 0.0;
  for (int64_t jc = j0; jc < j1; jc += 64) {
    const int cnt = (int)min<int64_t>(64, j1 - jc);
    if (lane < cnt) xr[wv][lane] = x[R[jc + lane]];
    wave_lds_sync();
    if (i < ns) {
#pragma unroll 8
      for (int j = 0; j < cnt; ++j) acc = fma(U12[(jc + j) * ns + i], xr[wv][j], acc);
    }
    wave_lds_sync();   // every lane's reads of this chunk before the next chunk overwrites it
  }
  part[wv][lane] = acc;
  __syncthreads();
  if (wv == 0 && i < ns)
    vbuf[s.voff + i] = x[s.first + i] - (((part[0][lane] + part[1][lane]) + part[2][lane]) + part[3][lane]);
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

// wrk[i] = Rs[p0[i]] * b[p0[i]]
__global__ void k_perm_in(int64_t n, const int64_t* __restrict__ p0, const double* __restrict__ Rs,
                          const double* __restrict__ b, double* __restrict__ wrk) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    int64_t r = p0[i];
    wrk[i] = Rs[r] * b[r];
  }
}
// x[q[i]] = wrk[i]
__global__ void k_perm_out(int64_t n, const int64_t* __restrict__ q, const double* __restrict__ wrk,
                           double* __restrict__ x) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[q[i]] = wrk[i];
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
// column order, deterministic), max |r_i| into *nrm; x += d.
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_residual(int64_t n, const int64_t* __restrict__ rowptr,
                                                  const int32_t* __restrict__ ent,
                                                  const int32_t* __restrict__ acol,
                                                  const double* __restrict__ a,
                                                  const double* __restrict__ x,
                                                  const double* __restrict__ b, double* __restrict__ r,
                                                  double* __restrict__ nrm) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  double ri = 0.0;
  if (i < n) {
    double acc = 0.0;
    for (int64_t e = rowptr[i]; e < rowptr[i + 1]; ++e) {
      const int32_t k = ent[e];
      acc = fma(a[k], x[acol[k]], acc);
    }
    ri = b[i] - acc;
    r[i] = ri;
  }
  const double m = wave_max(fabs(ri));
  if ((threadIdx.x & 63) == 0 && m > 0.0) atomic_max_pos(nrm, m);
}
__global__ void k_axpy1(int64_t n, const double* __restrict__ d, double* __restrict__ x) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[i] += d[i];
}

// ------------------------------------------------------------------------------------
// Host-side launch wrappers (called from smlu.cpp)
// ------------------------------------------------------------------------------------
static inline unsigned nblk(int64_t n, int b) { return (unsigned)((n + b - 1) / b); }
hipError_t launch_fwd(hipStream_t st, int cnt, const int32_t* list, const SNode* sn,
                      const int32_t* chlist, const int32_t* relmap, const int32_t* rowperm,
                      const double* store, double* x, double* vbuf) {
  if (cnt <= 0) return hipSuccess;
  k_fwd_front<<<cnt, 256, 0, st>>>(list, sn, chlist, relmap, rowperm, store, x, vbuf);
  return hipGetLastError();
}
hipError_t launch_bwd(hipStream_t st, int cnt, const int32_t* list, const SNode* sn,
                      const int32_t* rows, const double* store, double* x, double* vbuf) {
  if (cnt <= 0) return hipSuccess;
  k_bwd_front<<<cnt, 256, 0, st>>>(list, sn, rows, store, x, vbuf);
  return hipGetLastError();
}
hipError_t launch_fwd_gather(hipStream_t st, int cnt, const int32_t* list, const SNode* sn,
                             const int32_t* chlist, const int32_t* relmap, const int32_t* rowperm,
                             double* x, double* vbuf) {
  if (cnt <= 0) return hipSuccess;
  k_fwd_gather<<<cnt, 256, 0, st>>>(list, sn, chlist, relmap, rowperm, x, vbuf);
  return hipGetLastError();
}
hipError_t launch_tri_block(hipStream_t st, bool upper, int64_t nwg, const FrontTile* ft, int nft,
                            int step, const SNode* sn, const double* store, double* x, double* vbuf) {
  if (nwg <= 0) return hipSuccess;
  if (upper) k_tri_block<true><<<(unsigned)nwg, 320, 0, st>>>(ft, nft, step, sn, store, x, vbuf);
  else k_tri_block<false><<<(unsigned)nwg, 320, 0, st>>>(ft, nft, step, sn, store, x, vbuf);
  return hipGetLastError();
}
hipError_t launch_bwd_u12(hipStream_t st, int64_t nwg, const FrontTile* ft, int nft, const SNode* sn,
                          const int32_t* rows, const double* store, const double* x, double* vbuf) {
  if (nwg <= 0) return hipSuccess;
  k_bwd_u12<<<(unsigned)nwg, 256, 0, st>>>(ft, nft, sn, rows, store, x, vbuf);
  return hipGetLastError();
}
hipError_t launch_residual(hipStream_t st, int64_t n, const int64_t* rowptr, const int32_t* ent,
                           const int32_t* acol, const double* a, const double* x, const double* b,
                           double* r, double* nrm) {
  if (n <= 0) return hipSuccess;
  k_residual<<<nblk(n, 256), 256, 0, st>>>(n, rowptr, ent, acol, a, x, b, r, nrm);
  return hipGetLastError();
}
hipError_t launch_axpy1(hipStream_t st, int64_t n, const double* d, double* x) {
  if (n <= 0) return hipSuccess;
  k_axpy1<<<nblk(n, 256), 256, 0, st>>>(n, d, x);
  return hipGetLastError();
}
hipError_t launch_perm_in(hipStream_t st, int64_t n, const int64_t* p0, const double* Rs,
                          const double* b, double* wrk) {
  k_perm_in<<<nblk(n, 256), 256, 0, st>>>(n, p0, Rs, b, wrk);
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

hipError_t launch_perm_out(hipStream_t st, int64_t n, const int64_t* q, const double* wrk, double* x) {
  k_perm_out<<<nblk(n, 256), 256, 0, st>>>(n, q, wrk, x);
  return hipGetLastError();
}
hipError_t launch_unswap(hipStream_t st, int64_t n, const int64_t* pos_first, const int32_t* rowperm,
                         const double* in, double* out) {
  k_unswap<<<nblk(n, 256), 256, 0, st>>>(n, pos_first, rowperm, in, out);
  return hipGetLastError();
}


}  // namespace smlu
