// kernels_front.hip — gfx950 (CDNA4) kernels of the multifrontal numeric refactorization:
// assembly (scaling, scatter, extend-add), small fronts in LDS, and the latency-bound panel
// chain of the blocked large-front path.  The dense Schur updates are in kernels_gemm.hip
// (fp64 MFMA by default), the solves in kernels_solve.hip.
//
// Reference mapping (SharedMemSparseLU.jl):
//   k_rowscale            UMFPACK SUM scaling behind lu(A) (src/SharedMemSparseLU.jl:74, Rs at :51)
//   k_assemble            gather A's values into fronts (the "active columns") and the children's
//                         Schur-complement updates (extend-add), one pass per front column
//   k_front_lds           whole small fronts in LDS: pivot search, pivot scaling, rank-1 updates
//   k_panel_reg, k_laswp, the same column-elimination loop of lu(A)/lu!(F,A) (:74, :247) for
//   k_step_trsm, k_trsm_u, large fronts, blocked: panel, row swaps, triangular solves and
//   k_gemm*               Schur-complement (trailing) updates
//   k_fwd_front, k_tri_block, k_fwd_gather   lsolve! (:349-367)
//   k_bwd_front, k_bwd_u12                    rsolve! (:374-392)
#include "kernels_common.hpp"

namespace smlu {

// ------------------------------------------------------------------------------------
// Row scaling: Rs[i] = 1/sum_j |a_ij| summed in column order (bitwise equal to the oracle).
// ------------------------------------------------------------------------------------
// Entries eight at a time: the eight entry ids, then the eight values in flight together, then
// summed in order (one latency chain per eight entries instead of two per entry).
__global__ void k_rowscale(int64_t n, const int64_t* __restrict__ rowptr,
                           const int32_t* __restrict__ ent, const double* __restrict__ a,
                           double* __restrict__ Rs) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double s = 0.0;
  const int64_t e1 = rowptr[i + 1];
  for (int64_t e0 = rowptr[i]; e0 < e1; e0 += 8) {
    int32_t id[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) id[k] = e0 + k < e1 ? ent[e0 + k] : -1;
    double v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = id[k] >= 0 ? a[id[k]] : 0.0;
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (id[k] >= 0) s += fabs(v[k]);
  }
  Rs[i] = s > 0.0 ? 1.0 / s : 1.0;
}

__global__ void k_fill(int64_t n, double* __restrict__ x, double v) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[i] = v;
}

// Start of a factorization: info words and the growth maximum cleared, the local row permutation
// reset to the identity (rowperm = rowperm0) -- one kernel instead of memset / memcpy graph nodes.
__global__ void k_factor_reset(int64_t nnodes, int32_t* __restrict__ info, double* __restrict__ growth, int64_t n,
                               int32_t* __restrict__ rowperm, const int32_t* __restrict__ rowperm0) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nnodes) info[i] = 0;
  if (i < n) rowperm[i] = rowperm0[i];
  if (i == 0) growth[0] = 0.0;
}

// ------------------------------------------------------------------------------------
// Front assembly (one wave per front column, one launch per level): the column is built in
// 256-row chunks in LDS -- zeros, then the scaled A entries (plain stores: every entry owns
// its slot), then each contributing child's F22 column added in child order -- and written
// once, coalesced.  No memset of the fronts and no read-modify-write of the parent: every
// front element is written exactly once per factorization, every child F22 element and its
// row map read from HBM once (a chunk loads a child's row-map window and its values together;
// values whose rows fall in the next chunk are read again from L2).  The order of the additions per element is that of a zeroed front with
// A stored and the children added in child order (deterministic, no atomics).
// Lane q < 64 keeps the running position of contribution q in its child column (row maps are
// ascending, chunks are visited in ascending row order); contributions beyond the 64th find
// their start by binary search.
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_assemble(int64_t ntasks, const XCol* __restrict__ cols,
                                                  const XContrib* __restrict__ contrib,
                                                  const int2* __restrict__ aents,
                                                  const SNode* __restrict__ sn,
                                                  const int32_t* __restrict__ relmap,
                                                  const double* __restrict__ a,
                                                  const int32_t* __restrict__ arow,
                                                  const double* __restrict__ Rs,
                                                  double* __restrict__ store, double* __restrict__ scratch) {
  __shared__ double sbuf[4][256];
  const int64_t w = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (w >= ntasks) return;
  double* b = sbuf[threadIdx.x >> 6];
  const XCol t = cols[w];
  const SNode p = sn[t.p];
  FrontPtrs P = front_ptrs(p, store, scratch);
  const int64_t len = P.M;
  const int64_t tj = t.tj;
  // destination of local row r of this column
  gdbl* colL = tj < P.ns ? P.L + tj * P.M : nullptr;
  gdbl* colU = tj < P.ns ? nullptr : P.U + (tj - P.ns) * P.ns;
  gdbl* colF = (tj < P.ns || P.nu == 0) ? nullptr : P.F + (tj - P.ns) * P.nu - P.ns;
  // contribution q < 64: its descriptor lives in lane q for the whole column (read once),
  // together with its running position; each chunk then costs one row-map round trip (the
  // chunk's at most 256 entries of that child column are a prefix of the next 256) and one
  // round trip for the values it takes
  int cur = 0;                  // lane q: position in contribution q's child column
  int64_t q_src = 0, q_rm = 0;
  int q_nu = 0;
  if (lane < t.cnt) {
    const XContrib ck = contrib[t.off + lane];
    const SNode c = sn[ck.child];
    q_src = ck.src;
    q_rm = c.rowptr;
    q_nu = c.nu;
  }
  int64_t ap = 0;               // next A entry
  for (int64_t r0 = 0; r0 < len; r0 += 256) {
    const int64_t r1 = min<int64_t>(len, r0 + 256);
#pragma unroll
    for (int u = 0; u < 4; ++u) b[lane + 64 * u] = 0.0;
    wave_lds_sync();
    while (ap < t.acnt) {       // A entries with rows in [r0, r1): a prefix of the rest
      const int64_t i = ap + lane;
      int2 en = make_int2(0, 0x7fffffff);
      if (i < t.acnt) en = aents[t.aoff + i];
      const bool take = en.y < r1;
      const unsigned long long m = __ballot(take);
      if (take) b[en.y - r0] = Rs[arow[en.x]] * a[en.x];
      const int c = __popcll(m);
      ap += c;
      if (c < 64) break;
    }
    wave_lds_sync();
    for (int q = 0; q < t.cnt; ++q) {
      int64_t srco, rmo, nuc, pos;
      if (q < 64) {
        srco = ((int64_t)__builtin_amdgcn_readlane((int)(q_src >> 32), q) << 32) |
               (uint32_t)__builtin_amdgcn_readlane((int)(q_src & 0xffffffff), q);
        rmo = ((int64_t)__builtin_amdgcn_readlane((int)(q_rm >> 32), q) << 32) |
              (uint32_t)__builtin_amdgcn_readlane((int)(q_rm & 0xffffffff), q);
        nuc = __builtin_amdgcn_readlane(q_nu, q);
        pos = __builtin_amdgcn_readlane(cur, q);
      } else {                  // binary search for the first row >= r0
        const XContrib ck = contrib[t.off + q];
        const SNode c = sn[ck.child];
        srco = ck.src;
        rmo = c.rowptr;
        nuc = c.nu;
        const int32_t* rmq = relmap + rmo;
        int64_t lo = 0, hi = nuc;
        while (lo < hi) {
          const int64_t mid = (lo + hi) >> 1;
          if (rmq[mid] < r0) lo = mid + 1;
          else hi = mid;
        }
        pos = lo;
      }
      const double* src = srco >= 0 ? scratch + srco : store + (-1 - srco);
      const int32_t* rm = relmap + rmo;
      // row map and values in one round trip: the values are loaded for the whole window, the
      // ones whose rows fall beyond this chunk are read again by the next (from L2)
      int32_t rv[4];
      double sv[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int64_t i = pos + lane + 64 * k;
        rv[k] = i < nuc ? rm[i] : 0x7fffffff;
        sv[k] = i < nuc ? src[i] : 0.0;
      }
      int cn = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const bool take = rv[k] < r1;
        if (take) b[rv[k] - r0] += sv[k];
        cn += __popcll(__ballot(take));
      }
      pos += cn;
      if (q < 64 && lane == q) cur = (int)pos;
      wave_lds_sync();
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t r = r0 + lane + 64 * u;
      if (r < r1) {
        const double v = b[lane + 64 * u];
        if (colL) colL[r] = v;
        else if (r < P.ns) colU[r] = v;
        else colF[r] = v;
      }
    }
    wave_lds_sync();
  }
}

// ------------------------------------------------------------------------------------
// Pivot choice shared by the LDS and panel kernels: threshold partial pivoting with a
// diagonal preference (UMFPACK-style): keep the diagonal when |a_kk| >= diag_tol*amax.
// ------------------------------------------------------------------------------------
__device__ __forceinline__ int choose_pivot(double akk, double amax, int arg, int k,
                                            double diag_tol) {
  if (amax == 0.0) return k;
  if (fabs(akk) >= diag_tol * amax && akk != 0.0) return k;
  return arg;
}

// ------------------------------------------------------------------------------------
// Small fronts (M <= 128), assembly fused with the factorization: the whole front is built in
// LDS (zeros, the scaled A entries, each child's F22 block added in child order -- per element
// the order k_assemble uses), factored there, and written to L / U12 / F22 once; the front
// never makes an HBM round trip between assembly and factorization, and the small fronts need
// no k_assemble columns.  One workgroup of NW waves per front (NW = 1 for M <= 32, 2 for
// M <= 64, 4 above).  Right-looking partial LU over the ns fully-summed columns with pivot
// search over the fully-summed rows; the trailing F22 block receives its Schur update in the
// same pass.  list: (front, first A entry, A entry count) per front; A entries as (entry id,
// local column << 16 | local row).  The growth maximum is reduced over the front's columns and
// reported once.
// ------------------------------------------------------------------------------------
typedef double f64x4 __attribute__((ext_vector_type(4)));
template <int NW>
__global__ __launch_bounds__(64 * NW) void k_front_small(const int32_t* __restrict__ list,
                                                         const SNode* __restrict__ sn,
                                                         const int32_t* __restrict__ chlist,
                                                         const int32_t* __restrict__ relmap,
                                                         const int2* __restrict__ aents,
                                                         const double* __restrict__ a,
                                                         const int32_t* __restrict__ arow,
                                                         const double* __restrict__ Rs,
                                                         double* __restrict__ store,
                                                         double* __restrict__ scratch,
                                                         int32_t* __restrict__ rowperm,
                                                         int32_t* __restrict__ info,
                                                         double* __restrict__ growth, double diag_tol,
                                                         double piv_tol) {
  constexpr int NT = 64 * NW;
  extern __shared__ __attribute__((aligned(16))) double lds[];
  __shared__ int s_perm[128];
  __shared__ int s_piv;
  const int sid = list[3 * blockIdx.x];
  const int64_t a0 = list[3 * blockIdx.x + 1];
  const int acnt = list[3 * blockIdx.x + 2];
  const SNode s = sn[sid];
  FrontPtrs f = front_ptrs(s, store, scratch);
  const int M = (int)f.M, ns = (int)f.ns;
  const int ld = M | 1;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  // assembly
  for (int e = tid; e < M * ld; e += NT) lds[e] = 0.0;
  for (int i = tid; i < ns; i += NT) s_perm[i] = i;
  __syncthreads();
  for (int e = tid; e < acnt; e += NT) {
    const int2 en = aents[a0 + e];
    lds[(en.y >> 16) * ld + (en.y & 0xffff)] = Rs[arow[en.x]] * a[en.x];
  }
  __syncthreads();
  // children's F22 blocks, added in child order (a barrier between children): the lane's two rows
  // of the child's row map are read once per child, and a wave's columns go eight at a time --
  // their column indices and values all in flight before the first LDS addition
  for (int q = s.chbeg; q < s.chend; ++q) {
    const SNode c = sn[chlist[q]];
    const int nuc = c.nu;   // <= M <= 128: two rows per lane
    if (nuc == 0) continue;
    const int32_t* rm = relmap + c.rowptr;
    const gdbl* src = gbl(scratch + c.Foff);
    const bool h0 = lane < nuc, h1 = lane + 64 < nuc;
    const int ri0 = h0 ? rm[lane] : 0, ri1 = h1 ? rm[lane + 64] : 0;
    for (int jc0 = wv; jc0 < nuc; jc0 += 8 * NW) {
      int cj[8];
      double v0[8], v1[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int jc = jc0 + u * NW;
        const bool on = jc < nuc;
        cj[u] = on ? rm[jc] : 0;
        v0[u] = (on && h0) ? src[(int64_t)jc * nuc + lane] : 0.0;
        v1[u] = (on && h1) ? src[(int64_t)jc * nuc + lane + 64] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if (jc0 + u * NW >= nuc) break;
        double* col = lds + cj[u] * ld;
        if (h0) col[ri0] += v0[u];
        if (h1) col[ri1] += v1[u];
      }
    }
    __syncthreads();
  }
  // factorization
  int flag = 0, err = -1;   // wave 0, lane 0
  double gmax = 0.0, glane = 0.0;   // growth: lane 0 of wave 0 (full searches), per lane of wave 0 (fast ones)
  __shared__ int s_second;   // pair rule: position of the current pair's other row
  for (int k = 0; k < ns; ++k) {
    if (s.cpair && wv == 0) {   // ComplexF64 real-equivalent: pair-preserving pivots (mf.c rule)
      if ((k & 1) == 0) {
        double am = -1.0, amo = 0.0;
        int ai = k;
        for (int e = k + 2 * lane; e < M; e += 128) {
          const double x = lds[k * ld + e], y = lds[k * ld + e + 1];
          const double v = fma(x, x, y * y);
          if (e < ns) {
            if (v > am) { am = v; ai = e; }
          } else if (v > amo) {
            amo = v;
          }
        }
        am = wave_max_idx(am, ai);
        amo = wave_max(amo);
        if (lane == 0) {
          const double x = lds[k * ld + k], y = lds[k * ld + k + 1];
          const double d2 = fma(x, x, y * y);
          int pc = k;
          if (am <= 0.0) {
            flag |= 1;
            if (err < 0) err = k;
          } else if (!(d2 >= diag_tol * diag_tol * am && d2 != 0.0)) {
            pc = ai;
          }
          const int r1 = fabs(lds[k * ld + pc + 1]) > fabs(lds[k * ld + pc]) ? pc + 1 : pc;
          const int r2 = 2 * pc + 1 - r1;
          if (am > 0.0) {
            const double a = lds[k * ld + pc], b = lds[k * ld + pc + 1];
            const double pm = fma(a, a, b * b);
            if (pm < piv_tol * piv_tol * fmax(am, amo)) flag |= 2;
            gmax = fmax(gmax, sqrt(fmax(am, amo) / pm));
          }
          s_piv = r1;
          s_second = r2 == k ? r1 : r2;
        }
      } else if (lane == 0) {
        s_piv = s_second;
        if (lds[k * ld + s_second] == 0.0) {   // read before the swap: the row that moves to k
          flag |= 1;
          if (err < 0) err = k;
        }
      }
    } else if (wv == 0) {
      double am = -1.0, amo = 0.0;
      int ai = k;
      bool beats = false, weak = false;
      const double akk = lds[k * ld + k], pk = fabs(akk);
      for (int i = k + lane; i < M; i += 64) {
        double v = fabs(lds[k * ld + i]);
        if (i < ns) {
          if (v > am) { am = v; ai = i; }
          beats |= diag_tol * v > pk;
        } else if (v > amo) {
          amo = v;
        }
        weak |= piv_tol * v > pk;
      }
      // the diagonal stays unless a candidate beats it by 1/diag_tol (choose_pivot): one ballot
      // decides, and the weak-pivot test and the growth need no reduction either -- a product
      // or quotient by one positive number is monotone, so the per-lane maxima give the values
      // of the full reduction exactly (growth: each lane's max(|a_ik|)/|a_kk|, reduced at the end)
      if (akk != 0.0 && __ballot(beats) == 0ull) {
        const double ml = fmax(am, amo);
        if (ml > 0.0) glane = fmax(glane, ml / pk);
        const bool anyweak = __ballot(weak) != 0ull;
        if (lane == 0) {
          if (anyweak) flag |= 2;
          s_piv = k;
        }
        goto searched;
      }
      am = wave_max_idx(am, ai);
      amo = wave_max(amo);
      if (lane == 0) {
        int piv = choose_pivot(lds[k * ld + k], am, ai, k, diag_tol);
        double pv = fabs(lds[k * ld + piv]);
        if (am <= 0.0) {
          flag |= 1;
          if (err < 0) err = k;
        } else {
          if (pv < piv_tol * fmax(am, amo)) flag |= 2;
          gmax = fmax(gmax, fmax(am, amo) / pv);
        }
        s_piv = piv;
      }
    }
  searched:
    __syncthreads();
    const int piv = s_piv;
    if (piv != k) {
      for (int j = tid; j < M; j += NT) {
        double t = lds[j * ld + k];
        lds[j * ld + k] = lds[j * ld + piv];
        lds[j * ld + piv] = t;
      }
      if (tid == 0) {
        int t = s_perm[k];
        s_perm[k] = s_perm[piv];
        s_perm[piv] = t;
      }
      __syncthreads();
    }
    const double pinv = recip(lds[k * ld + k]);
    for (int i = k + 1 + tid; i < M; i += NT) lds[k * ld + i] = lds[k * ld + i] * pinv;
    __syncthreads();
    // Schur update of the pivot block and the U12 rows only; F22 (rows and columns >= ns) takes
    // all ns rank-1 updates at once after the loop, on the matrix cores.  Wave jobs: U12 column
    // groups (lanes over 64 columns, rows (k, ns) in a loop) and the pivot columns (k, ns) (lanes
    // over the rows (k, M)), dealt round-robin.  Per element the same fma as the rank-1 pass over
    // the whole front, skipped when u == 0.
    const int nb = (M - ns + 63) / 64, nl = ns - k - 1;
    for (int q = wv; q < nb + nl; q += NW) {
      if (q < nb) {
        const int j = ns + 64 * q + lane;
        if (j < M) {
          double* cj = lds + j * ld;
          const double u = cj[k];
          if (u != 0.0) {
            int i = k + 1;
            for (; i + 4 <= ns; i += 4) {
              const double a0 = cj[i], a1 = cj[i + 1], a2 = cj[i + 2], a3 = cj[i + 3];
              const double l0 = lds[k * ld + i], l1 = lds[k * ld + i + 1], l2 = lds[k * ld + i + 2],
                           l3 = lds[k * ld + i + 3];
              cj[i] = fma(-l0, u, a0);
              cj[i + 1] = fma(-l1, u, a1);
              cj[i + 2] = fma(-l2, u, a2);
              cj[i + 3] = fma(-l3, u, a3);
            }
            for (; i < ns; ++i) cj[i] = fma(-lds[k * ld + i], u, cj[i]);
          }
        }
      } else {
        const int j = k + 1 + (q - nb);
        const double u = lds[j * ld + k];
        if (u != 0.0)
          for (int i = k + 1 + lane; i < M; i += 64)
            lds[j * ld + i] = fma(-lds[k * ld + i], u, lds[j * ld + i]);
      }
    }
    __syncthreads();
  }
  // F22 -= L21 * U12 with k = ns on the fp64 matrix cores, 16 x 16 output blocks dealt to the
  // waves: C starts as the block's F22 values, A = -L21 (rows ns.., k-quads of the pivot
  // columns), B = U12; per element the ns products are fused in ascending k, as the rank-1 pass
  // did (which skipped u == 0: the two differ only in the sign of an exactly zero entry).
  if (M > ns) {
    const int nu = M - ns, nt = (nu + 15) / 16;
    const int li = lane & 15, lg = lane >> 4;
    for (int t = wv; t < nt * nt; t += NW) {
      const int r0 = ns + 16 * (t % nt), c0 = ns + 16 * (t / nt);
      const int ra = r0 + li, cb = c0 + li;
      f64x4 acc;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = r0 + lg + 4 * r;
        acc[r] = (i < M && cb < M) ? lds[cb * ld + i] : 0.0;
      }
      for (int kq = 0; kq < ns; kq += 4) {
        const int kk = kq + lg;
        const double fa = (kk < ns && ra < M) ? -lds[kk * ld + ra] : 0.0;
        const double fb = (kk < ns && cb < M) ? lds[cb * ld + kk] : 0.0;
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(fa, fb, acc, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = r0 + lg + 4 * r;
        if (i < M && cb < M) lds[cb * ld + i] = acc[r];
      }
    }
    __syncthreads();
  }
  // store: L panel, U12 and F22 are each one contiguous column-major block
  for (int j = wv; j < M; j += NW) {
    for (int i = lane; i < M; i += 64) *fel(f, i, j) = lds[j * ld + i];
  }
  for (int i = tid; i < ns; i += NT) rowperm[s.first + i] = s_perm[i];
  if (wv == 0) gmax = fmax(gmax, wave_max(glane));
  if (tid == 0) {
    if (flag) publish_info(info + sid, flag, err);
    if (gmax > 0.0) atomic_max_pos(&growth[0], gmax);
  }
}



// ------------------------------------------------------------------------------------
// Panel factorization with the candidate rows in REGISTERS: thread t owns candidate row t
// (R <= 64*NW) as row[0..W).  No physical row swaps: pos[t] is the row's current position
// (LAPACK transposition semantics, so at most 2w rows move); who[] maps positions to threads.
// Per column k: the diagonal candidate (position k) is accepted when no other candidate
// exceeds |a_kk|/diag_tol (one ballot per wave); only otherwise a full argmax runs.  The
// pivot row is broadcast through LDS; each thread updates its own row in registers.
// ------------------------------------------------------------------------------------
template <int W, int NW>
__global__ __launch_bounds__(64 * NW) void k_panel_reg(const int32_t* __restrict__ list, int step,
                                                       const SNode* __restrict__ sn,
                                                       double* __restrict__ store,
                                                       double* __restrict__ scratch,
                                                       int32_t* __restrict__ rowperm,
                                                       int32_t* __restrict__ swaps,
                                                       int64_t swap_stride,
                                                       int32_t* __restrict__ info,
                                                       double* __restrict__ growth, double diag_tol) {
  static_assert(W == 32 || W == 64, "panel width");
  __shared__ __attribute__((aligned(16))) double s_prow[64];
  __shared__ int s_who[64 * NW];
  __shared__ int s_old[64 * NW];
  __shared__ double s_val[NW];
  __shared__ int s_idx[NW];
  __shared__ int s_any[NW];
  __shared__ int s_piv;
  __shared__ double s_cv[64 * NW];            // pair rule: the column's values by position
  int second = 0;                             // pair rule: position of the pair's other row
  const int sid = list[2 * blockIdx.x];       // (front, swap slot) pairs
  const SNode s = sn[sid];
  FrontPtrs f = front_ptrs(s, store, scratch);
  const int64_t M = f.M;
  const int ns = (int)f.ns;
  const int kb = step * s.nb;
  const int w = min(s.nb, ns - kb);
  const int R = (s.mode == 1) ? ns - kb : w;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const bool has = tid < R;
  gdbl* P = f.L + (int64_t)kb * M + kb;
  double rA[32], rB[32];   // columns [0,32) and [32,64) of my candidate row
#pragma unroll
  for (int j = 0; j < 32; ++j) {
    rA[j] = (has && j < w) ? P[(int64_t)j * M + tid] : 0.0;
    rB[j] = (W == 64 && has && j + 32 < w) ? P[(int64_t)(j + 32) * M + tid] : 0.0;
  }
  int pos = tid;
  s_who[tid] = tid;
  int flag = 0, err = -1;
  double lmax = 0.0;
  __syncthreads();
  // one elimination step at panel column kabs; `cur` holds that column at index kk, `rest`
  // (when RESTB) is the whole second half that is updated too
  // the pivot-candidate lane writes its row halves with 16-byte LDS stores (entries left of
  // the current column are written too; nobody reads them in this step)
  auto publish = [&](double (&cur)[32], double (&rest)[32], const int base, const bool restb) {
    double2* d = reinterpret_cast<double2*>(s_prow + base);
#pragma unroll
    for (int j = 0; j < 16; ++j) d[j] = make_double2(cur[2 * j], cur[2 * j + 1]);
    if (restb) {
      double2* d2 = reinterpret_cast<double2*>(s_prow + 32);
#pragma unroll
      for (int j = 0; j < 16; ++j) d2[j] = make_double2(rest[2 * j], rest[2 * j + 1]);
    }
  };
  auto column = [&](double (&cur)[32], double (&rest)[32], const int kk, const int kabs,
                    const bool restb) {
    const int q = s_who[kabs];
    const bool cand = has && pos >= kabs;
    // optimistic: the diagonal candidate publishes its whole row (the pivot row if accepted)
    if (tid == q) publish(cur, rest, kabs - kk, restb);
    if (s.cpair && (kabs & 1) == 0 && has) s_cv[pos] = cur[kk];
    __syncthreads();
    const double akk = s_prow[kabs];
    int p = q;
    if (s.cpair) {   // ComplexF64 real-equivalent: pair-preserving pivots (oracle/mf.c rule)
      if ((kabs & 1) == 0) {
        const double pv = has ? s_cv[pos ^ 1] : 0.0;
        const double m2 = fma(cur[kk], cur[kk], pv * pv);
        const bool lead = cand && (pos & 1) == 0;
        double am = lead ? m2 : -1.0;
        int ai = lead ? pos : 0x7fffffff;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
          const double ov = __shfl_xor(am, o, 64);
          const int oi = __shfl_xor(ai, o, 64);
          if (ov > am || (ov == am && oi < ai)) { am = ov; ai = oi; }
        }
        if (NW > 1) {
          if (lane == 0) { s_val[wv] = am; s_idx[wv] = ai; }
          __syncthreads();
          am = s_val[0];
          ai = s_idx[0];
#pragma unroll
          for (int v = 1; v < NW; ++v)
            if (s_val[v] > am || (s_val[v] == am && s_idx[v] < ai)) { am = s_val[v]; ai = s_idx[v]; }
        }
        const double x = s_cv[kabs], y = s_cv[kabs + 1];
        const double d2 = fma(x, x, y * y);
        int pc = kabs;
        if (am <= 0.0) {
          flag |= 1;
          if (err < 0) err = kb + kabs;
        } else if (!(d2 >= diag_tol * diag_tol * am && d2 != 0.0)) {
          pc = ai;
        }
        const int r1 = fabs(s_cv[pc + 1]) > fabs(s_cv[pc]) ? pc + 1 : pc;
        const int r2 = 2 * pc + 1 - r1;
        second = r2 == kabs ? r1 : r2;
        p = s_who[r1];
      } else {
        p = s_who[second];
      }
      if (p != q) {             // publish the chosen pivot row
        __syncthreads();
        if (tid == p) {
          publish(cur, rest, kabs - kk, restb);
          s_piv = pos;
        }
        __syncthreads();
      }
      if ((kabs & 1) == 1 && s_prow[kabs] == 0.0) {
        flag |= 1;
        if (err < 0) err = kb + kabs;
      }
    } else {
    const bool beats = cand && pos != kabs && fabs(cur[kk]) * diag_tol > fabs(akk);
    bool any = __ballot(beats) != 0ull;
    if (NW > 1) {
      if (lane == 0) s_any[wv] = any ? 1 : 0;
      __syncthreads();
      any = false;
#pragma unroll
      for (int v = 0; v < NW; ++v) any |= s_any[v] != 0;
    }
    if (any || akk == 0.0) {   // full argmax over the candidates (rare under dominance)
      double am = cand ? fabs(cur[kk]) : -1.0;
      int ai = cand ? pos : 0x7fffffff;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const double ov = __shfl_xor(am, o, 64);
        const int oi = __shfl_xor(ai, o, 64);
        if (ov > am || (ov == am && oi < ai)) { am = ov; ai = oi; }
      }
      if (NW > 1) {
        if (lane == 0) { s_val[wv] = am; s_idx[wv] = ai; }
        __syncthreads();
        am = s_val[0];
        ai = s_idx[0];
#pragma unroll
        for (int v = 1; v < NW; ++v)
          if (s_val[v] > am || (s_val[v] == am && s_idx[v] < ai)) { am = s_val[v]; ai = s_idx[v]; }
      }
      if (am <= 0.0) {
        flag |= 1;
        if (err < 0) err = kb + kabs;
      } else {
        p = s_who[ai];
      }
      if (p != q) {             // re-publish the chosen pivot row
        __syncthreads();
        if (tid == p) {
          publish(cur, rest, kabs - kk, restb);
          s_piv = pos;
        }
        __syncthreads();
      }
    }
    }
    const double pinv = recip(s_prow[kabs]);
    if (cand && tid != p) {
      const double l = cur[kk] * pinv;
      cur[kk] = l;
      lmax = fmax(lmax, fabs(l));
      if (l != 0.0) {
        // pivot-row reads batched ahead of their FMAs (one LDS latency per half-row)
        double pr[32];
#pragma unroll
        for (int j = 0; j < 32; ++j)
          if (j > kk) pr[j] = s_prow[kabs - kk + j];
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < 32; ++j)
          if (j > kk) cur[j] = fma(-l, pr[j], cur[j]);
        __builtin_amdgcn_sched_barrier(0);
        if (restb) {
#pragma unroll
          for (int j = 0; j < 32; ++j) pr[j] = s_prow[32 + j];
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int j = 0; j < 32; ++j) rest[j] = fma(-l, pr[j], rest[j]);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    }
    if (p != q) {               // transposition of positions kabs and ppos
      const int ppos = s_piv;
      if (tid == p) pos = kabs;
      else if (tid == q) pos = ppos;
      __syncthreads();
      if (tid == 0) {
        s_who[kabs] = p;
        s_who[ppos] = q;
      }
    }
    __syncthreads();
  };
#pragma unroll
  for (int k = 0; k < 32; ++k)
    if (k < w) column(rA, rB, k, k, W == 64 && w > 32);
  if (W == 64) {
#pragma unroll
    for (int k = 0; k < 32; ++k)
      if (k + 32 < w) column(rB, rA, k, k + 32, false);
  }
  if (has) {
#pragma unroll
    for (int j = 0; j < 32; ++j) {
      if (j < w) P[(int64_t)j * M + pos] = rA[j];
      if (W == 64 && j + 32 < w) P[(int64_t)(j + 32) * M + pos] = rB[j];
    }
  }
  int32_t* rp = rowperm + s.first + kb;
  if (has) s_old[tid] = rp[tid];
  __syncthreads();
  if (has) rp[pos] = s_old[tid];
  int32_t* sw = swaps + (int64_t)list[2 * blockIdx.x + 1] * swap_stride;
  const bool mv = has && pos != tid;
  const unsigned long long m = __ballot(mv);
  if (lane == 0) s_any[wv] = __popcll(m);
  __syncthreads();
  int base = 0;
  for (int v = 0; v < wv; ++v) base += s_any[v];
  if (mv) {
    const int o = base + __popcll(m & ((1ull << lane) - 1ull));
    sw[1 + 2 * o] = pos;
    sw[2 + 2 * o] = tid;
  }
  if (tid == 0) {
    int tot = 0;
    for (int v = 0; v < NW; ++v) tot += s_any[v];
    sw[0] = tot;
  }
  lmax = wave_max(lmax);
  if (lane == 0) s_val[wv] = lmax;
  __syncthreads();
  if (tid == 0) {
    double g = 0.0;
    for (int v = 0; v < NW; ++v) g = fmax(g, s_val[v]);
    if (g > 0.0) atomic_max_pos(&growth[0], g);
    if (flag) publish_info(info + sid, flag, err);
  }
}

// Single-wave variant of k_panel_reg (R <= 64 candidate rows): the same pivot choices and the
// same arithmetic, with every broadcast done by v_readlane from the owning lane instead of
// through LDS -- no LDS traffic and no barriers on the per-column chain.  who (position ->
// thread) is kept one entry per lane.

template <int W>
__global__ __launch_bounds__(64) void k_panel_wave(const int32_t* __restrict__ list, int step,
                                                   const SNode* __restrict__ sn,
                                                   double* __restrict__ store,
                                                   double* __restrict__ scratch,
                                                   int32_t* __restrict__ rowperm,
                                                   int32_t* __restrict__ swaps,
                                                   int64_t swap_stride,
                                                   int32_t* __restrict__ info,
                                                   double* __restrict__ growth, double diag_tol) {
  static_assert(W == 32 || W == 64, "panel width");
  const int sid = list[2 * blockIdx.x];
  const SNode s = sn[sid];
  FrontPtrs f = front_ptrs(s, store, scratch);
  const int64_t M = f.M;
  const int ns = (int)f.ns;
  const int kb = step * s.nb;
  const int w = min(s.nb, ns - kb);
  const int R = (s.mode == 1) ? ns - kb : w;
  const int lane = threadIdx.x;
  const bool has = lane < R;
  gdbl* P = f.L + (int64_t)kb * M + kb;
  double rA[32], rB[32];
#pragma unroll
  for (int j = 0; j < 32; ++j) {
    rA[j] = (has && j < w) ? P[(int64_t)j * M + lane] : 0.0;
    rB[j] = (W == 64 && has && j + 32 < w) ? P[(int64_t)(j + 32) * M + lane] : 0.0;
  }
  int pos = lane, who = lane;
  int flag = 0, err = -1;
  double lmax = 0.0;
  int second = 0;   // pair rule: position of the current pair's other row
  auto column = [&](double (&cur)[32], double (&rest)[32], const int kk, const int kabs,
                    const bool restb) {
    const int q = __builtin_amdgcn_readfirstlane(__builtin_amdgcn_readlane(who, kabs));
    const bool cand = has && pos >= kabs;
    const double akk = readlane_f64(cur[kk], q);
    int p = q;
    if (s.cpair) {   // ComplexF64 real-equivalent: pair-preserving pivots (oracle/mf.c rule)
      if ((kabs & 1) == 0) {
        const int plane = __shfl(who, pos ^ 1, 64);          // lane holding my pair partner
        const double pv = __shfl(cur[kk], plane, 64);
        const double m2 = fma(cur[kk], cur[kk], pv * pv);
        const bool lead = cand && (pos & 1) == 0;
        double am = lead ? m2 : -1.0;
        int ai = lead ? pos : 0x7fffffff;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
          const double ov = __shfl_xor(am, o, 64);
          const int oi = __shfl_xor(ai, o, 64);
          if (ov > am || (ov == am && oi < ai)) { am = ov; ai = oi; }
        }
        const double d2 = readlane_f64(m2, q);
        int pc = kabs;
        if (am <= 0.0) {
          flag |= 1;
          if (err < 0) err = kb + kabs;
        } else if (!(d2 >= diag_tol * diag_tol * am && d2 != 0.0)) {
          pc = __builtin_amdgcn_readfirstlane(ai);
        }
        const double va = readlane_f64(cur[kk], __builtin_amdgcn_readlane(who, pc));
        const double vb = readlane_f64(cur[kk], __builtin_amdgcn_readlane(who, pc + 1));
        const int r1 = fabs(vb) > fabs(va) ? pc + 1 : pc;
        const int r2 = 2 * pc + 1 - r1;
        second = r2 == kabs ? r1 : r2;
        p = __builtin_amdgcn_readfirstlane(__builtin_amdgcn_readlane(who, r1));
      } else {
        p = __builtin_amdgcn_readfirstlane(__builtin_amdgcn_readlane(who, second));
        if (readlane_f64(cur[kk], p) == 0.0) {
          flag |= 1;
          if (err < 0) err = kb + kabs;
        }
      }
    } else if (__ballot(cand && pos != kabs && fabs(cur[kk]) * diag_tol > fabs(akk)) != 0ull || akk == 0.0) {
      // full argmax (rare under dominance)
      double am = cand ? fabs(cur[kk]) : -1.0;
      int ai = cand ? pos : 0x7fffffff;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const double ov = __shfl_xor(am, o, 64);
        const int oi = __shfl_xor(ai, o, 64);
        if (ov > am || (ov == am && oi < ai)) { am = ov; ai = oi; }
      }
      if (am <= 0.0) {
        flag |= 1;
        if (err < 0) err = kb + kabs;
      } else {
        p = __builtin_amdgcn_readlane(who, __builtin_amdgcn_readfirstlane(ai));
      }
      p = __builtin_amdgcn_readfirstlane(p);
    }
    const double pinv = recip(readlane_f64(cur[kk], p));
    if (cand && lane != p) {
      const double l = cur[kk] * pinv;
      cur[kk] = l;
      lmax = fmax(lmax, fabs(l));
      if (l != 0.0) {
#pragma unroll
        for (int j = 0; j < 32; ++j)
          if (j > kk) cur[j] = fma(-l, readlane_f64(cur[j], p), cur[j]);
        if (restb) {
#pragma unroll
          for (int j = 0; j < 32; ++j) rest[j] = fma(-l, readlane_f64(rest[j], p), rest[j]);
        }
      }
    }
    if (p != q) {               // transposition of positions kabs and ppos
      const int ppos = __builtin_amdgcn_readlane(pos, p);
      if (lane == p) pos = kabs;
      else if (lane == q) pos = ppos;
      if (lane == kabs) who = p;
      else if (lane == ppos) who = q;
    }
  };
#pragma unroll
  for (int k = 0; k < 32; ++k)
    if (k < w) column(rA, rB, k, k, W == 64 && w > 32);
  if (W == 64) {
#pragma unroll
    for (int k = 0; k < 32; ++k)
      if (k + 32 < w) column(rB, rA, k, k + 32, false);
  }
  if (has) {
#pragma unroll
    for (int j = 0; j < 32; ++j) {
      if (j < w) P[(int64_t)j * M + pos] = rA[j];
      if (W == 64 && j + 32 < w) P[(int64_t)(j + 32) * M + pos] = rB[j];
    }
  }
  int32_t* rp = rowperm + s.first + kb;
  const int old = has ? rp[lane] : 0;
  if (has) rp[pos] = old;
  int32_t* sw = swaps + (int64_t)list[2 * blockIdx.x + 1] * swap_stride;
  const bool mv = has && pos != lane;
  const unsigned long long m = __ballot(mv);
  if (mv) {
    const int o = __popcll(m & ((1ull << lane) - 1ull));
    sw[1 + 2 * o] = pos;
    sw[2 + 2 * o] = lane;
  }
  if (lane == 0) sw[0] = __popcll(m);
  lmax = wave_max(lmax);
  if (lane == 0) {
    if (lmax > 0.0) atomic_max_pos(&growth[0], lmax);
    if (flag) publish_info(info + sid, flag, err);
  }
}

typedef double v4d __attribute__((ext_vector_type(4)));
// Dev instrumentation (-DSMLU_PANEL_TRACE, tools/panel_trace.py): workgroup 0 of every fused panel
// launch records the 100 MHz clock at its phase boundaries.  The product build has no hook.
#ifdef SMLU_PANEL_TRACE
struct PanelTrace {
  long long* buf;
  unsigned long long* ctr;
  long long n;
};
__device__ PanelTrace g_panel_trace;
__device__ __forceinline__ void pmark(long long idx, int k) {
  if (idx >= 0 && threadIdx.x == 0) g_panel_trace.buf[idx * 16 + k] = (long long)__builtin_amdgcn_s_memrealtime();
}
#define PMARK(k) pmark(s_pidx, k)
// slots 8..15: shader-clock cycles (s_memtime) at the hand-off of blocks 7 and 8 between waves:
// owner start / owner end (before the barrier) / next wave past the barrier / next wave applied
__device__ __forceinline__ void pmarkc(long long idx, int k, bool who) {
  if (idx >= 0 && who && (threadIdx.x & 63) == 0) g_panel_trace.buf[idx * 16 + k] = (long long)__builtin_amdgcn_s_memtime();
}
#define PMARKB(blk, k, who) \
  do { if ((blk) == 7 || (blk) == 8) pmarkc(s_pidx, 8 + 4 * ((blk) - 7) + (k), (who)); } while (0)
#else
#define PMARK(k) ((void)0)
#define PMARKB(blk, k, who) ((void)0)
#endif
// Tail of the fused panel (k_panel_blk<NWV, true>): the finished tile (x, row positions pos)
// goes to LDS as k_tri_inv reads it from HBM ([col][row], ld 65, identity outside w x w), wave v
// forms columns 4v..4v+3 of NL = I - L^-1 and of NU = I - U^-1 with k_tri_inv's arithmetic, and
// the outer block's other columns [ostart, oend) \ [kb, kb+w) get the tile's row interchanges
// (every moved row read into registers, one barrier, then written to its new position).
template <int NWV, int CW, bool INV>
__device__ __forceinline__ void panel_fused_tail(const double (&x)[CW], int pos, bool has, int w, int kb,
                                                 int64_t M, const FrontPtrs& f, const SNode& s, int64_t slot,
                                                 double* __restrict__ tinv, int ob, int lane, int wv,
                                                 long long s_pidx) {
  (void)s_pidx;
  static_assert((NWV == 16 && CW == 4) || (NWV == 8 && CW == 8), "fused panel: 16 x 4 or 8 x 8 columns");
  __shared__ double sD[INV ? 64 * 65 : 1];
  const int tid = threadIdx.x;
  if (INV) {
    for (int idx = tid; idx < 4096; idx += 64 * NWV) {
      const int i = idx & 63, j = idx >> 6;
      if (i >= w || j >= w) sD[j * 65 + i] = i == j ? 1.0 : 0.0;
    }
    if (has) {
#pragma unroll
      for (int j = 0; j < CW; ++j) {
        const int c = wv * CW + j;
        if (c < w) sD[c * 65 + pos] = x[j];
      }
    }
  }
  // row interchanges of the outer block's other columns: read every moved row first
  const int ostart = (kb / ob) * ob, oend = min((int)f.ns, ostart + ob);
  const int nother = oend - ostart - w;
  const bool moved = has && pos != lane;
  constexpr int kMaxCols = 320 / NWV;   // (OB - 64) / NWV columns per wave for OB <= 384
  double mv[kMaxCols];
#pragma unroll
  for (int q = 0; q < kMaxCols; ++q) {
    const int cj = wv + NWV * q;
    if (moved && cj < nother) {
      const int col = ostart + cj + (ostart + cj >= kb ? w : 0);
      mv[q] = f.L[(int64_t)col * M + kb + lane];
    }
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < kMaxCols; ++q) {
    const int cj = wv + NWV * q;
    if (moved && cj < nother) {
      const int col = ostart + cj + (ostart + cj >= kb ? w : 0);
      f.L[(int64_t)col * M + kb + pos] = mv[q];
    }
  }
  PMARK(3);
  if (!INV) return;
  // tile inverses X_L = L^-1, X_U = U^-1 by 16 x 16 blocks: the diagonal blocks by substitution
  // (lane = one column of one block), the off-diagonal blocks by the block recurrences
  //   X_ij = -X_ii sum_{k=j}^{i-1} L_ik X_kj (i > j),   X_ij = -X_ii sum_{k=i+1}^{j} U_ik X_kj (i < j)
  // on the fp64 matrix cores (distance 1, 2, 3 from the diagonal, one barrier each); then
  // NL = I - X_L, NU = I - X_U to the tinv slot (the operands of the GEMM-form TRSM launches).
  __shared__ double XL[64 * 65], XU[64 * 65];   // [col][row], ld 65
  const int li = lane & 15, lg = lane >> 4;
  if (wv < 2) {   // wave 0: the four L diagonal blocks, wave 1: the four U diagonal blocks
    const int b0 = 16 * lg, c = li;
    double xv[16];
    if (wv == 0) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        double v = i == c ? 1.0 : 0.0;
#pragma unroll
        for (int j = 0; j < i; ++j) v = fma(-sD[(b0 + j) * 65 + b0 + i], xv[j], v);
        xv[i] = v;
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) XL[(b0 + c) * 65 + b0 + i] = xv[i];
    } else {
#pragma unroll
      for (int i = 15; i >= 0; --i) {
        double v = i == c ? 1.0 : 0.0;
#pragma unroll
        for (int j = i + 1; j < 16; ++j) v = fma(-sD[(b0 + j) * 65 + b0 + i], xv[j], v);
        xv[i] = v * recip(sD[(b0 + i) * 65 + b0 + i]);
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) XU[(b0 + c) * 65 + b0 + i] = xv[i];
    }
  }
  __syncthreads();
  PMARK(4);
  // one off-diagonal block (bi, bj) at distance d: T = sum_k F_{bi,k} X_{k,bj}, X = -X_{bi,bi} T.
  // MFMA 16x16x4: A fragment lane (row li, k lg), B fragment (k lg, col li); D lane holds
  // (row lg + 4r, col li), which is exactly the B fragment of k-quad r for the second product.
  auto offdiag = [&](const double* X, double* Xw, int bi, int bj, int k0, int k1) {
    v4d t = {0.0, 0.0, 0.0, 0.0};
    for (int kb = k0; kb <= k1; ++kb) {
#pragma unroll
      for (int kq = 0; kq < 4; ++kq) {
        const double fa = sD[(16 * kb + 4 * kq + lg) * 65 + 16 * bi + li];   // F[bi rows][kb cols]
        const double fb = X[(16 * bj + li) * 65 + 16 * kb + 4 * kq + lg];    // X[kb rows][bj cols]
        t = __builtin_amdgcn_mfma_f64_16x16x4f64(fa, fb, t, 0, 0, 0);
      }
    }
    v4d x = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int kq = 0; kq < 4; ++kq) {
      const double fa = -X[(16 * bi + 4 * kq + lg) * 65 + 16 * bi + li];    // -X[bi rows][bi cols]
      x = __builtin_amdgcn_mfma_f64_16x16x4f64(fa, t[kq], x, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) Xw[(16 * bj + li) * 65 + 16 * bi + lg + 4 * r] = x[r];
  };
  for (int d = 1; d < 4; ++d) {
    const int nb = 4 - d;   // blocks at distance d: L (j + d, j), U (j, j + d), j < nb
    if (wv < nb) offdiag(XL, XL, wv + d, wv, wv, wv + d - 1);
    else if (wv >= NWV / 2 && wv - NWV / 2 < nb)
      offdiag(XU, XU, wv - NWV / 2, wv - NWV / 2 + d, wv - NWV / 2 + 1, wv - NWV / 2 + d);
    __syncthreads();
  }
  PMARK(5);
  double* out = tinv + slot * 8192;
  for (int idx = tid; idx < 4096; idx += 64 * NWV) {
    const int i = idx & 63, j = idx >> 6;
    out[(int64_t)j * 64 + i] = i > j ? -XL[j * 65 + i] : 0.0;
    out[4096 + (int64_t)j * 64 + i] = i == j ? 1.0 - XU[j * 65 + i] : (i < j ? -XU[j * 65 + i] : 0.0);
  }
}

// Column-block panel (the 64-wide panels; round 2's per-column-barrier variant k_panel_cols was
// dropped in round 4): wave w owns the
// CW = 64/NWV consecutive columns [w*CW, (w+1)*CW) in registers (lane = candidate row).  The
// owner of a block factors its CW columns wave-locally -- pivot search, scaling, rank-1 updates
// of its own later columns, no workgroup barrier -- and publishes the block's pivots and
// multipliers through LDS (double-buffered); after ONE barrier every later wave applies the CW
// rank-1 updates to its columns in column order, and every wave replays the transpositions.
// One barrier per CW columns instead of one per column.  Same pivot choices and the same
// element-wise FMAs in the same order as k_panel_wave (bitwise-identical panel).
//
// FUSED = true (GEMM-form fronts, nb = 64): the same panel, then in the same workgroup the two
// tile inverses k_tri_inv computes (same per-column arithmetic: bitwise-identical NL/NU in the
// same tinv slot) and the row interchanges of the outer block's other columns that k_laswp
// applies inside the block -- two launches fewer per inner step of the blocked fronts.
template <int NWV, int FUSED>
__global__ __launch_bounds__(64 * NWV) void k_panel_blk(const int32_t* __restrict__ list, int step,
                                                        const SNode* __restrict__ sn,
                                                        double* __restrict__ store,
                                                        double* __restrict__ scratch,
                                                        int32_t* __restrict__ rowperm,
                                                        int32_t* __restrict__ swaps,
                                                        int64_t swap_stride,
                                                        int32_t* __restrict__ info,
                                                        double* __restrict__ growth, double diag_tol,
                                                        double* __restrict__ tinv, int ob) {
  constexpr int CW = 64 / NWV;
  __shared__ double s_l[2][CW][64];
  __shared__ int s_p[2][CW];
  __shared__ int s_flag[NWV], s_err[NWV];
  __shared__ double s_gmax[NWV];
#ifdef SMLU_PANEL_TRACE
  __shared__ long long s_pidx_sh;
  if (threadIdx.x == 0)
    s_pidx_sh = (blockIdx.x == 0 && g_panel_trace.buf) ? (long long)atomicAdd(g_panel_trace.ctr, 1ull) : -1;
  __syncthreads();
  const long long s_pidx = s_pidx_sh < (g_panel_trace.n) ? s_pidx_sh : -1;
#else
  const long long s_pidx = -1;
#endif
  PMARK(0);
  const int sid = list[2 * blockIdx.x];
  const SNode s = sn[sid];
  FrontPtrs f = front_ptrs(s, store, scratch);
  const int64_t M = f.M;
  const int ns = (int)f.ns;
  const int kb = step * s.nb;
  const int w = min(s.nb, ns - kb);
  const int R = (s.mode == 1) ? ns - kb : w;
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool has = lane < R;
  gdbl* P = f.L + (int64_t)kb * M + kb;
  double x[CW];
#pragma unroll
  for (int j = 0; j < CW; ++j) {
    const int c = wv * CW + j;
    x[j] = (has && c < w) ? P[(int64_t)c * M + lane] : 0.0;
  }
  int pos = lane, who = lane;   // replicated in every wave
  int flag = 0, err = -1;
  double lmax = 0.0;
  auto transpose = [&](int k, int p, int q) {   // positions k and pos[p] exchange rows
    if (p != q) {
      const int ppos = __builtin_amdgcn_readlane(pos, p);
      if (lane == p) pos = k;
      else if (lane == q) pos = ppos;
      if (lane == k) who = p;
      else if (lane == ppos) who = q;
    }
  };
  PMARK(1);
  for (int blk = 0; blk < NWV; ++blk) {
    const int k0 = blk * CW;
    if (k0 >= w) break;
    const int buf = blk & 1;
    if (wv == blk) {   // the owner factors its block
      PMARKB(blk, 0, true);
#pragma unroll
      for (int j = 0; j < CW; ++j) {
        const int k = k0 + j;
        if (k < w) {
          const int q = __builtin_amdgcn_readfirstlane(__builtin_amdgcn_readlane(who, k));
          const double cur = x[j];
          const bool cand = has && pos >= k;
          const double akk = readlane_f64(cur, q);
          // the reciprocal of the diagonal candidate starts at once (the usual pivot; its
          // dependent fp64 chain overlaps the candidate test)
          double pinv = recip(akk);
          const bool beats = cand && pos != k && fabs(cur) * diag_tol > fabs(akk);
          int p = q;
          if (__ballot(beats) != 0ull || akk == 0.0) {   // full argmax (rare under dominance)
            double am = cand ? fabs(cur) : -1.0;
            int ai = cand ? pos : 0x7fffffff;
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
              const double ov = __shfl_xor(am, o, 64);
              const int oi = __shfl_xor(ai, o, 64);
              if (ov > am || (ov == am && oi < ai)) { am = ov; ai = oi; }
            }
            if (am <= 0.0) {
              flag |= 1;
              if (err < 0) err = kb + k;
            } else {
              p = __builtin_amdgcn_readlane(who, __builtin_amdgcn_readfirstlane(ai));
            }
            p = __builtin_amdgcn_readfirstlane(p);
            pinv = recip(readlane_f64(cur, p));
          }
          double l = 0.0;
          if (cand && lane != p) {
            l = cur * pinv;
            lmax = fmax(lmax, fabs(l));
            x[j] = l;
          }
          s_l[buf][j][lane] = l;
          if (lane == 0) s_p[buf][j] = p;
          if (l != 0.0) {
#pragma unroll
            for (int j2 = j + 1; j2 < CW; ++j2) x[j2] = fma(-l, readlane_f64(x[j2], p), x[j2]);
          }
          transpose(k, p, q);
        }
      }
      PMARKB(blk, 1, true);
    }
    __syncthreads();
    PMARKB(blk, 2, wv == blk + 1);
    if (wv != blk) {   // later waves apply the block's updates; every wave replays the swaps
      // the block's pivots and multipliers in one LDS round trip (not one pair per column)
      int pj[CW];
      double lj[CW];
#pragma unroll
      for (int j = 0; j < CW; ++j) {
        pj[j] = s_p[buf][j];
        lj[j] = s_l[buf][j][lane];
      }
#pragma unroll
      for (int j = 0; j < CW; ++j) {
        const int k = k0 + j;
        if (k < w) {
          const int q = __builtin_amdgcn_readfirstlane(__builtin_amdgcn_readlane(who, k));
          const int p = __builtin_amdgcn_readfirstlane(pj[j]);
          if (wv > blk) {
            const double l = lj[j];
            if (l != 0.0) {
#pragma unroll
              for (int jj = 0; jj < CW; ++jj) x[jj] = fma(-l, readlane_f64(x[jj], p), x[jj]);
            }
          }
          transpose(k, p, q);
        }
      }
      PMARKB(blk, 3, wv == blk + 1);
    }
  }
  if (has) {
#pragma unroll
    for (int j = 0; j < CW; ++j) {
      const int c = wv * CW + j;
      if (c < w) P[(int64_t)c * M + pos] = x[j];
    }
  }
  PMARK(2);
  lmax = wave_max(lmax);
  if (lane == 0) {
    s_gmax[wv] = lmax;
    s_flag[wv] = flag;
    s_err[wv] = err;
  }
  if constexpr (FUSED > 0)
    panel_fused_tail<NWV, CW, FUSED == 2>(x, pos, has, w, kb, M, f, s, list[2 * blockIdx.x + 1], tinv, ob, lane, wv,
                                          s_pidx);
  __syncthreads();
  PMARK(6);
  if (wv == 1 && lane == 0) {   // the growth maximum (a read, maybe an atomic) beside wave 0's bookkeeping
    double g = 0.0;
    for (int v = 0; v < NWV; ++v) g = fmax(g, s_gmax[v]);
    if (g > 0.0) atomic_max_pos(&growth[0], g);
  }
  if (wv != 0) return;
  int32_t* rp = rowperm + s.first + kb;
  const int old = has ? rp[lane] : 0;
  if (has) rp[pos] = old;
  int32_t* sw = swaps + (int64_t)list[2 * blockIdx.x + 1] * swap_stride;
  const bool mv = has && pos != lane;
  const unsigned long long m = __ballot(mv);
  if (mv) {
    const int o = __popcll(m & ((1ull << lane) - 1ull));
    sw[1 + 2 * o] = pos;
    sw[2 + 2 * o] = lane;
  }
  if (lane == 0) {
    sw[0] = __popcll(m);
    int fl = 0, er = -1;
    for (int v = 0; v < NWV; ++v) {   // first failing column over all waves
      fl |= s_flag[v];
      if (s_err[v] >= 0 && (er < 0 || s_err[v] < er)) er = s_err[v];
    }
    if (fl) publish_info(info + sid, fl, er);
  }
  PMARK(7);
}

#ifdef SMLU_PANEL_TRACE
// Dev hook for tools/panel_trace.py: n > 0 arms the trace for the next n fused panel launches;
// n == 0 copies the records (16 clock values per launch) out and disarms it.
extern "C" int smlu_dev_panel_trace(long long n, long long* out) {
  static long long* buf = nullptr;
  static unsigned long long* ctr = nullptr;
  static long long cap = 0;
  using namespace smlu;
  PanelTrace t{nullptr, nullptr, 0};
  if (n > 0) {
    if (buf) (void)hipFree(buf);
    if (!ctr && hipMalloc(&ctr, sizeof(unsigned long long)) != hipSuccess) return -1;
    if (hipMalloc(&buf, sizeof(long long) * 16 * n) != hipSuccess) return -1;
    (void)hipMemset(buf, 0, sizeof(long long) * 16 * n);
    (void)hipMemset(ctr, 0, sizeof(unsigned long long));
    cap = n;
    t = PanelTrace{buf, ctr, n};
  } else if (buf) {
    (void)hipDeviceSynchronize();
    if (out && hipMemcpy(out, buf, sizeof(long long) * 16 * cap, hipMemcpyDeviceToHost) != hipSuccess) return -1;
  }
  return hipMemcpyToSymbol(HIP_SYMBOL(g_panel_trace), &t, sizeof t) == hipSuccess ? 0 : -1;
}
#endif


// Row swaps (LAPACK laswp) of the panels of a SwapTask on its column set; one workgroup per 64
// columns.  Within a workgroup the panels' swap lists are applied in order.  A list moves at
// most 64 rows (mode 1 panels are 32 wide, mode 2 pivots inside the 64-row diagonal tile);
// a panel without swaps costs one load.
__device__ __forceinline__ int find_swap_task(const SwapTask* __restrict__ t, int cnt, int64_t b) {
  int lo = 0, hi = cnt - 1;
  while (lo < hi) {
    int mid = (lo + hi + 1) >> 1;
    if (t[mid].wg0 <= b) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// ------------------------------------------------------------------------------------
// Full-candidate panel for tall candidate sets (mode 1, R > 512 rows: the re-pivoting
// refactor puts every blocked front in mode 1).  One 1024-thread workgroup per front works on
// the panel in place in HBM/L2 (the candidates do not fit in registers): per column the same
// diagonal-preference test and argmax (ties to the lowest position) as k_panel_reg, a
// physical swap of the two rows across the w panel columns, then scaling and the rank-1
// update of the remaining panel columns by rows.  The transpositions are turned into the
// (final position, original offset) swap list and the rowperm update the other kernels use.
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void k_panel_tall(const int32_t* __restrict__ list, int step,
                                                     const SNode* __restrict__ sn,
                                                     double* __restrict__ store,
                                                     double* __restrict__ scratch,
                                                     int32_t* __restrict__ rowperm,
                                                     int32_t* __restrict__ swaps,
                                                     int64_t swap_stride,
                                                     int32_t* __restrict__ info,
                                                     double* __restrict__ growth, double diag_tol) {
  constexpr int NT = 1024, NWV = NT / 64;
  __shared__ double s_val[NWV];
  __shared__ int s_idx[NWV];
  __shared__ int s_any[NWV];
  __shared__ int s_tp[64];          // transposition partner of each panel column
  __shared__ int s_key[128], s_org[128];
  __shared__ int32_t s_rp[128];
  const int sid = list[2 * blockIdx.x];
  const SNode s = sn[sid];
  FrontPtrs f = front_ptrs(s, store, scratch);
  const int64_t M = f.M;
  const int ns = (int)f.ns;
  const int kb = step * s.nb;
  const int w = min(s.nb, ns - kb);
  const int R = (s.mode == 1) ? ns - kb : w;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  gdbl* P = f.L + (int64_t)kb * M + kb;
  int flag = 0, err = -1;
  double lmax = 0.0;
  int second = 0;   // pair rule: position of the current pair's other row
  for (int k = 0; k < w; ++k) {
    gdbl* col = P + (int64_t)k * M;
    const double akk = col[k];
    if (s.cpair) {   // ComplexF64 real-equivalent: pair-preserving pivots (oracle/mf.c rule)
      int p;
      if ((k & 1) == 0) {
        double am = -1.0;
        int ai = 0x7fffffff;
        for (int e = k + 2 * tid; e < R; e += 2 * NT) {
          const double v = fma(col[e], col[e], col[e + 1] * col[e + 1]);
          if (v > am) { am = v; ai = e; }
        }
        am = wave_max_idx(am, ai);
        if (lane == 0) { s_val[wv] = am; s_idx[wv] = ai; }
        __syncthreads();
        am = s_val[0];
        ai = s_idx[0];
        for (int v = 1; v < NWV; ++v)
          if (s_val[v] > am || (s_val[v] == am && s_idx[v] < ai)) { am = s_val[v]; ai = s_idx[v]; }
        const double d2 = fma(col[k], col[k], col[k + 1] * col[k + 1]);
        int pc = k;
        if (am <= 0.0) {
          flag |= 1;
          if (err < 0) err = kb + k;
        } else if (!(d2 >= diag_tol * diag_tol * am && d2 != 0.0)) {
          pc = ai;
        }
        const int r1 = fabs(col[pc + 1]) > fabs(col[pc]) ? pc + 1 : pc;
        const int r2 = 2 * pc + 1 - r1;
        second = r2 == k ? r1 : r2;
        p = r1;
      } else {
        p = second;
        if (col[p] == 0.0) {
          flag |= 1;
          if (err < 0) err = kb + k;
        }
      }
      __syncthreads();   // every thread has read the column before the interchange
      if (tid == 0) s_tp[k] = p;
      if (p != k) {
        for (int j = tid; j < w; j += NT) {
          const double a = P[(int64_t)j * M + k];
          P[(int64_t)j * M + k] = P[(int64_t)j * M + p];
          P[(int64_t)j * M + p] = a;
        }
      }
      __syncthreads();
      const double pinv = recip(col[k]);
      for (int r = k + 1 + tid; r < R; r += NT) {
        const double l = col[r] * pinv;
        col[r] = l;
        lmax = fmax(lmax, fabs(l));
        if (l != 0.0)
          for (int j = k + 1; j < w; ++j) P[(int64_t)j * M + r] = fma(-l, P[(int64_t)j * M + k], P[(int64_t)j * M + r]);
      }
      __syncthreads();
      continue;
    }
    bool beats = false;
    for (int r = k + 1 + tid; r < R; r += NT) beats |= fabs(col[r]) * diag_tol > fabs(akk);
    const bool any_w = __ballot(beats) != 0ull;
    if (lane == 0) s_any[wv] = any_w ? 1 : 0;
    __syncthreads();
    bool any = false;
    for (int v = 0; v < NWV; ++v) any |= s_any[v] != 0;
    int p = k;
    if (any || akk == 0.0) {
      double am = -1.0;
      int ai = 0x7fffffff;
      for (int r = k + tid; r < R; r += NT) {
        const double v = fabs(col[r]);
        if (v > am) { am = v; ai = r; }   // rows visited in increasing order: ties keep the lowest
      }
      am = wave_max_idx(am, ai);
      if (lane == 0) { s_val[wv] = am; s_idx[wv] = ai; }
      __syncthreads();
      am = s_val[0];
      ai = s_idx[0];
      for (int v = 1; v < NWV; ++v)
        if (s_val[v] > am || (s_val[v] == am && s_idx[v] < ai)) { am = s_val[v]; ai = s_idx[v]; }
      if (am <= 0.0) {
        flag |= 1;
        if (err < 0) err = kb + k;
      } else {
        p = ai;
      }
    }
    if (tid == 0) s_tp[k] = p;
    if (p != k) {   // physical interchange of rows k and p across the panel columns
      for (int j = tid; j < w; j += NT) {
        const double a = P[(int64_t)j * M + k];
        P[(int64_t)j * M + k] = P[(int64_t)j * M + p];
        P[(int64_t)j * M + p] = a;
      }
    }
    __syncthreads();
    const double pinv = recip(col[k]);
    for (int r = k + 1 + tid; r < R; r += NT) {
      const double l = col[r] * pinv;
      col[r] = l;
      lmax = fmax(lmax, fabs(l));
      if (l != 0.0)
        for (int j = k + 1; j < w; ++j) P[(int64_t)j * M + r] = fma(-l, P[(int64_t)j * M + k], P[(int64_t)j * M + r]);
    }
    __syncthreads();
  }
  // net permutation of the touched positions: position -> original offset
  if (tid == 0) {
    int nk = 0;
    auto slot = [&](int x) {
      for (int i = 0; i < nk; ++i)
        if (s_key[i] == x) return i;
      s_key[nk] = x;
      s_org[nk] = x;
      return nk++;
    };
    for (int k = 0; k < w; ++k) {
      const int p = s_tp[k];
      if (p == k) continue;
      const int a = slot(k), b = slot(p);
      const int t = s_org[a];
      s_org[a] = s_org[b];
      s_org[b] = t;
    }
    int32_t* rp = rowperm + s.first + kb;
    for (int i = 0; i < nk; ++i) s_rp[i] = rp[s_org[i]];
    int32_t* sw = swaps + (int64_t)list[2 * blockIdx.x + 1] * swap_stride;
    int m = 0;
    for (int i = 0; i < nk; ++i) {
      if (s_key[i] == s_org[i]) continue;
      rp[s_key[i]] = s_rp[i];
      sw[1 + 2 * m] = s_key[i];
      sw[2 + 2 * m] = s_org[i];
      ++m;
    }
    sw[0] = m;
  }
  lmax = wave_max(lmax);
  if (lane == 0) s_val[wv] = lmax;
  __syncthreads();
  if (tid == 0) {
    double g = 0.0;
    for (int v = 0; v < NWV; ++v) g = fmax(g, s_val[v]);
    if (g > 0.0) atomic_max_pos(&growth[0], g);
    if (flag) publish_info(info + sid, flag, err);
  }
}

__global__ __launch_bounds__(256) void k_laswp(const SwapTask* __restrict__ tasks, int ntask,
                                               const SNode* __restrict__ sn,
                                               double* __restrict__ store,
                                               double* __restrict__ scratch,
                                               const int32_t* __restrict__ swaps, int64_t swap_stride) {
  __shared__ double buf[64 * 65];   // [column][moved row]
  const SwapTask t = tasks[find_swap_task(tasks, ntask, blockIdx.x)];
  const int64_t c0 = ((int64_t)blockIdx.x - t.wg0) * 64;
  const int64_t ntot = (int64_t)(t.b - t.a) - (t.c_hi - t.c_lo);
  const int ncol = (int)min<int64_t>(64, ntot - c0);
  if (ncol <= 0) return;
  const SNode s = sn[t.s];
  FrontPtrs f = front_ptrs(s, store, scratch);
  const int skip = t.c_hi - t.c_lo;
  for (int u = 0; u < t.nsub; ++u) {
    const int32_t* sw = swaps + (int64_t)(t.slot0 + u) * swap_stride;
    const int nsw = sw[0];
    if (nsw == 0) continue;   // uniform per workgroup
    const int kb = t.kb0 + u * s.nb;
    const int cnt = min(64, nsw);
    for (int idx = threadIdx.x; idx < cnt * ncol; idx += 256) {
      const int p = idx % cnt, cj = idx / cnt;
      int64_t col = t.a + c0 + cj;
      if (col >= t.c_lo) col += skip;
      buf[cj * 65 + p] = *fel(f, kb + sw[2 + 2 * p], col);
    }
    __syncthreads();
    for (int idx = threadIdx.x; idx < cnt * ncol; idx += 256) {
      const int p = idx % cnt, cj = idx / cnt;
      int64_t col = t.a + c0 + cj;
      if (col >= t.c_lo) col += skip;
      *fel(f, kb + sw[1 + 2 * p], col) = buf[cj * 65 + p];
    }
    __syncthreads();
  }
}


template <int W>
__global__ __launch_bounds__(256) void k_trsm_u(const FrontTile* __restrict__ ft, int nft, int OB,
                                                int mode, const SNode* __restrict__ sn,
                                                double* __restrict__ store,
                                                double* __restrict__ scratch,
                                                const int32_t* __restrict__ swaps,
                                                int64_t swap_stride) {
  // outer phase (mode 1): U rows [kb, kb+w) of the columns [oend, M), kb = FrontTile.pad;
  // one thread per column, the column in registers, L_kk broadcast from LDS
  (void)mode;
  (void)swaps;
  (void)swap_stride;
  __shared__ double sT[W * W];
  const int64_t b = blockIdx.x;
  const int fi = find_front_tile(ft, nft, b);
  const SNode s = sn[ft[fi].s];
  const int64_t tile = b - ft[fi].wg0;
  FrontPtrs f = front_ptrs(s, store, scratch);
  const int64_t M = f.M;
  const int ns = (int)f.ns;
  const int kb = ft[fi].pad;
  const int w = min(s.nb, ns - kb);
  const int64_t ostart = (int64_t)(kb / OB) * OB;
  const int64_t oend = min<int64_t>(ns, ostart + OB);
  const int tid = threadIdx.x;
  const gdbl* Lkk = f.L + (int64_t)kb * M + kb;
  for (int idx = tid; idx < W * W; idx += 256) {
    const int i = idx % W, j = idx / W;
    sT[idx] = (i < w && j < w) ? Lkk[(int64_t)j * M + i] : 0.0;
  }
  __syncthreads();
  const int64_t col = oend + tile * 256 + tid;
  if (col >= M) return;
  gdbl* cp = fel(f, kb, col);
  double x[W];
  if (w == W) {
#pragma unroll
    for (int j = 0; j < W; ++j) x[j] = cp[j];
    lower_unit_solve_fast<W>(x, sT);
#pragma unroll
    for (int j = 0; j < W; ++j) cp[j] = x[j];
    return;
  }
  if (W == 64 && w == 32) {   // 32-wide panels (mode 1 fronts)
#pragma unroll
    for (int j = 0; j < 32; ++j) x[j] = cp[j];
    lower_unit_solve_fast<32, W>(x, sT);
#pragma unroll
    for (int j = 0; j < 32; ++j) cp[j] = x[j];
    return;
  }
#pragma unroll
  for (int j = 0; j < W; ++j) x[j] = j < w ? cp[j] : 0.0;
#pragma unroll
  for (int j = 0; j < W; ++j) {
    if (j < w) {
      const double xj = x[j];
#pragma unroll
      for (int i = j + 1; i < W; ++i) x[i] = fma(-sT[j * W + i], xj, x[i]);
    }
  }
#pragma unroll
  for (int j = 0; j < W; ++j)
    if (j < w) cp[j] = x[j];
}


// ------------------------------------------------------------------------------------
// One launch per inner step for both triangular solves of the panel (row swaps already
// applied by k_laswp):
//   role U (workgroups [0, nU)): U[kb:kb+w, c] = L_kk^{-1} A[kb:kb+w, c] for the columns
//     c in [kb+w, oend) of the outer block, one thread per column, the column in registers,
//     L_kk broadcast from LDS;
//   role L (workgroups [nU, nU+nL)): rows below the candidate block, L = A U_kk^{-1}, one
//     thread per row in registers, U_kk broadcast from LDS; growth max for the threshold test.
// ------------------------------------------------------------------------------------
template <int W>
__global__ __launch_bounds__(256) void k_step_trsm(const FrontTile* __restrict__ ftU, int nftU, int64_t nU,
                                                   const FrontTile* __restrict__ ftL, int nftL,
                                                   int step, int OB, const SNode* __restrict__ sn,
                                                   double* __restrict__ store,
                                                   double* __restrict__ scratch,
                                                   int32_t* __restrict__ info,
                                                   double* __restrict__ growth, double piv_tol) {
  __shared__ double sT[W * W];   // L_kk (role U) or U_kk (role L), [col][row]
  __shared__ double s_rd[W];     // 1 / diag(U_kk) (role L)
  __shared__ double s_red[4];
  const int64_t b = blockIdx.x;
  const int tid = threadIdx.x;
  if (b < nU) {
    const int fi = find_front_tile(ftU, nftU, b);
    const SNode s = sn[ftU[fi].s];
    const int64_t tile = b - ftU[fi].wg0;
    FrontPtrs f = front_ptrs(s, store, scratch);
    const int64_t M = f.M;
    const int ns = (int)f.ns;
    const int kb = ftU[fi].pad;
    const int w = min(s.nb, ns - kb);
    const int64_t ostart = (int64_t)(kb / OB) * OB;
    const int64_t oend = min<int64_t>(ns, ostart + OB);
    const gdbl* Lkk = f.L + (int64_t)kb * M + kb;
    for (int idx = tid; idx < W * W; idx += 256) {
      const int i = idx % W, j = idx / W;
      sT[idx] = (i < w && j < w) ? Lkk[(int64_t)j * M + i] : 0.0;
    }
    __syncthreads();
    const int64_t col = kb + w + tile * 256 + tid;
    if (col < oend && w == W) {
      gdbl* cp = fel(f, kb, col);
      double x[W];
#pragma unroll
      for (int j = 0; j < W; ++j) x[j] = cp[j];
      lower_unit_solve_fast<W>(x, sT);
#pragma unroll
      for (int j = 0; j < W; ++j) cp[j] = x[j];
    } else if (col < oend) {
      gdbl* cp = fel(f, kb, col);   // rows [kb, kb+w) of this column are contiguous
      double x[W];
#pragma unroll
      for (int j = 0; j < W; ++j) x[j] = j < w ? cp[j] : 0.0;
      // the runtime guard splits the unrolled solve into per-step blocks; without it the
      // scheduler hoists all 2016 LDS reads into one block and spills
#pragma unroll
      for (int j = 0; j < W; ++j) {
        if (j < w) {
          const double xj = x[j];
#pragma unroll
          for (int i = j + 1; i < W; ++i) x[i] = fma(-sT[j * W + i], xj, x[i]);
        }
      }
#pragma unroll
      for (int j = 0; j < W; ++j)
        if (j < w) cp[j] = x[j];
    }
    return;
  }
  // role L
  const int64_t bl = b - nU;
  const int fi = find_front_tile(ftL, nftL, bl);
  const int sid = ftL[fi].s;
  const SNode s = sn[sid];
  const int64_t tile = bl - ftL[fi].wg0;
  FrontPtrs f = front_ptrs(s, store, scratch);
  const int64_t M = f.M;
  const int ns = (int)f.ns;
  const int kb = step * s.nb;
  const int w = min(s.nb, ns - kb);
  const int R = (s.mode == 1) ? ns - kb : w;
  const int64_t r0 = kb + R;
  gdbl* P = f.L + (int64_t)kb * M;
  for (int idx = tid; idx < W * W; idx += 256) {
    const int i = idx % W, j = idx / W;
    sT[idx] = (i < w && j < w) ? P[(int64_t)j * M + kb + i] : 0.0;
  }
  __syncthreads();
  if (tid < W) s_rd[tid] = tid < w ? recip(sT[tid * W + tid]) : 0.0;
  __syncthreads();
  const int64_t row = r0 + tile * 256 + tid;
  double gmax = 0.0;
  if (row < M && w == W) {
    double x[W];
#pragma unroll
    for (int j = 0; j < W; ++j) x[j] = P[(int64_t)j * M + row];
    gmax = upper_right_solve_fast<W>(x, sT, s_rd);
#pragma unroll
    for (int j = 0; j < W; ++j) P[(int64_t)j * M + row] = x[j];
  } else if (row < M) {
    double x[W];
#pragma unroll
    for (int j = 0; j < W; ++j) x[j] = (j < w) ? P[(int64_t)j * M + row] : 0.0;
#pragma unroll
    for (int j = 0; j < W; ++j) {
      if (j < w) {
        x[j] = x[j] * s_rd[j];
        gmax = fmax(gmax, fabs(x[j]));
#pragma unroll
        for (int k = j + 1; k < W; ++k) x[k] = fma(-x[j], sT[k * W + j], x[k]);
      }
    }
#pragma unroll
    for (int j = 0; j < W; ++j)
      if (j < w) P[(int64_t)j * M + row] = x[j];
  }
  gmax = wave_max(gmax);
  if ((tid & 63) == 0) s_red[tid >> 6] = gmax;
  __syncthreads();
  if (tid == 0) {
    const double g = fmax(fmax(s_red[0], s_red[1]), fmax(s_red[2], s_red[3]));
    if (g > 0.0) atomic_max_pos(&growth[0], g);
    if (g > 1.0 / piv_tol) atomicOr(&info[sid], 2);
  }
}


// ------------------------------------------------------------------------------------
// Host-side launch wrappers (called from smlu.cpp)
// ------------------------------------------------------------------------------------
static inline unsigned nblk(int64_t n, int b) { return (unsigned)((n + b - 1) / b); }

// Dynamic LDS above 64 KiB must be enabled per kernel before launch (and before any capture).
hipError_t init_kernel_attributes() {
  const void* fs[3] = {(const void*)k_front_small<1>, (const void*)k_front_small<2>, (const void*)k_front_small<4>};
  for (const void* k : fs) {
    hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t launch_rowscale(hipStream_t st, int64_t n, const int64_t* rowptr, const int32_t* ent,
                           const double* a, double* Rs) {
  if (n <= 0) return hipSuccess;
  k_rowscale<<<nblk(n, 256), 256, 0, st>>>(n, rowptr, ent, a, Rs);
  return hipGetLastError();
}
hipError_t launch_factor_reset(hipStream_t st, int64_t nnodes, int32_t* info, double* growth, int64_t n,
                               int32_t* rowperm, const int32_t* rowperm0) {
  const int64_t m = nnodes > n ? nnodes : (n > 1 ? n : 1);
  k_factor_reset<<<nblk(m, 256), 256, 0, st>>>(nnodes, info, growth, n, rowperm, rowperm0);
  return hipGetLastError();
}
hipError_t launch_fill(hipStream_t st, int64_t n, double* x, double v) {
  if (n <= 0) return hipSuccess;
  k_fill<<<nblk(n, 256), 256, 0, st>>>(n, x, v);
  return hipGetLastError();
}
hipError_t launch_assemble(hipStream_t st, int64_t ntasks, const XCol* cols, const XContrib* contrib,
                           const int2* aents, const SNode* sn, const int32_t* relmap, const double* a,
                           const int32_t* arow, const double* Rs, double* store, double* scratch) {
  if (ntasks <= 0) return hipSuccess;
  k_assemble<<<(unsigned)((ntasks + 3) / 4), 256, 0, st>>>(ntasks, cols, contrib, aents, sn, relmap, a, arow,
                                                            Rs, store, scratch);
  return hipGetLastError();
}
hipError_t launch_front_small(hipStream_t st, int cnt, int Mmax, const int32_t* list, const SNode* sn,
                              const int32_t* chlist, const int32_t* relmap, const int2* aents, const double* a,
                              const int32_t* arow, const double* Rs, double* store, double* scratch,
                              int32_t* rowperm, int32_t* info, double* growth, double diag_tol, double piv_tol) {
  if (cnt <= 0) return hipSuccess;
  if (Mmax > 128) return hipErrorInvalidValue;
  size_t lds = (size_t)Mmax * (size_t)(Mmax | 1) * sizeof(double);
#define FS_ARGS list, sn, chlist, relmap, aents, a, arow, Rs, store, scratch, rowperm, info, growth, diag_tol, piv_tol
  if (Mmax <= 32) k_front_small<1><<<cnt, 64, lds, st>>>(FS_ARGS);
  else if (Mmax <= 64) k_front_small<2><<<cnt, 128, lds, st>>>(FS_ARGS);
  else k_front_small<4><<<cnt, 256, lds, st>>>(FS_ARGS);
#undef FS_ARGS
  return hipGetLastError();
}
hipError_t launch_panel1(hipStream_t st, int cnt, int lds_doubles, int rmax, int wmax, int step,
                         const int32_t* list,
                         const SNode* sn, double* store, double* scratch, int32_t* rowperm,
                         int32_t* swaps, int64_t swap_stride, int32_t* info, double* growth,
                         double diag_tol, int fused, double* tinv, int ob) {
  if (cnt <= 0) return hipSuccess;
  size_t lds = (size_t)lds_doubles * sizeof(double);
#define PANEL1_ARGS list, step, sn, store, scratch, rowperm, swaps, swap_stride, info, growth, diag_tol
  (void)lds;
  if (fused) {   // GEMM-form fronts: panel + in-block row interchanges (+ tile inverses if fused == 2)
    if (wmax <= 32 || ob > 64 + 16 * 20 || (fused == 2 && !tinv)) return hipErrorInvalidValue;
    if (fused == 2) k_panel_blk<16, 2><<<cnt, 1024, 0, st>>>(PANEL1_ARGS, tinv, ob);
    else k_panel_blk<16, 1><<<cnt, 1024, 0, st>>>(PANEL1_ARGS, tinv, ob);
  }
  // 64-wide panels: the column-block kernel (16 waves, one barrier per 4 columns)
  else if (wmax > 32) k_panel_blk<16, 0><<<cnt, 1024, 0, st>>>(PANEL1_ARGS, nullptr, 0);
  // 32-wide panels (full-candidate fronts): one wave up to 64 rows, register tiles up to 512
  else if (rmax <= 64) k_panel_wave<32><<<cnt, 64, 0, st>>>(PANEL1_ARGS);
  else if (rmax <= 128) k_panel_reg<32, 2><<<cnt, 128, 0, st>>>(PANEL1_ARGS);
  else if (rmax <= 256) k_panel_reg<32, 4><<<cnt, 256, 0, st>>>(PANEL1_ARGS);
  else if (rmax <= 512) k_panel_reg<32, 8><<<cnt, 512, 0, st>>>(PANEL1_ARGS);
  else k_panel_tall<<<cnt, 1024, 0, st>>>(PANEL1_ARGS);   // full-candidate panels of the re-pivoting refactor
#undef PANEL1_ARGS
  return hipGetLastError();
}
hipError_t launch_laswp(hipStream_t st, int64_t nwg, const SwapTask* tasks, int ntask, const SNode* sn,
                        double* store, double* scratch, const int32_t* swaps, int64_t swap_stride) {
  if (nwg <= 0) return hipSuccess;
  k_laswp<<<(unsigned)nwg, 256, 0, st>>>(tasks, ntask, sn, store, scratch, swaps, swap_stride);
  return hipGetLastError();
}
hipError_t launch_step_trsm(hipStream_t st, int W, const FrontTile* ftU, int nftU, int64_t nU,
                            const FrontTile* ftL, int nftL, int64_t nL, int step, int OB, const SNode* sn,
                            double* store, double* scratch, int32_t* info, double* growth, double piv_tol) {
  if (nU + nL <= 0) return hipSuccess;
  if (W <= 32)
    k_step_trsm<32><<<(unsigned)(nU + nL), 256, 0, st>>>(ftU, nftU, nU, ftL, nftL, step, OB, sn, store,
                                                         scratch, info, growth, piv_tol);
  else
    k_step_trsm<64><<<(unsigned)(nU + nL), 256, 0, st>>>(ftU, nftU, nU, ftL, nftL, step, OB, sn, store,
                                                         scratch, info, growth, piv_tol);
  return hipGetLastError();
}
hipError_t launch_trsm_u(hipStream_t st, int64_t nwg, const FrontTile* ft, int nft, int OB, int mode,
                         const SNode* sn, double* store, double* scratch, const int32_t* swaps,
                         int64_t swap_stride) {
  if (nwg <= 0) return hipSuccess;
  k_trsm_u<64><<<(unsigned)nwg, 256, 0, st>>>(ft, nft, OB, mode, sn, store, scratch, swaps, swap_stride);
  return hipGetLastError();
}

}  // namespace smlu
