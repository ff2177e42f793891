// device.hpp — types shared by the host schedule (smlu.cpp) and the gfx950 kernels
// (kernels.hip).  One record per supernode (front) and one per GEMM region.
#pragma once
#include <cstdint>

namespace smlu {

// Front s is the dense M x M matrix (M = ns + nu) over index set [first, first+ns) U R_s.
// It lives in three column-major pieces:
//   columns [0, ns)            : L panel   store[Loff + j*M + i]        (ld M)
//   rows [0, ns),  cols >= ns  : U12       store[Uoff + (j-ns)*ns + i]  (ld ns)
//   rows >= ns,    cols >= ns  : F22       scratch[Foff + (j-ns)*nu + (i-ns)] (ld nu)
struct SNode {
  int64_t first;
  int64_t Loff, Uoff, Foff;   // Foff = -1 when nu == 0
  int64_t rowptr;             // into rows[] / relmap[] (nu entries)
  int64_t voff;               // front vector offset for the solves (M doubles)
  int32_t ns, nu;
  int32_t parent, nb;         // nb = panel width of the blocked path (0 = LDS path)
  int32_t mode;               // 0 = LDS front kernel, 1 = blocked + full-candidate pivoting,
                              // 2 = blocked + diagonal-tile pivoting with growth check
  int32_t chbeg, chend;       // children in chlist[chbeg, chend)
  int32_t level;
  int32_t cpair;              // 1: ComplexF64 real-equivalent, pair-preserving pivots (rows and
                              //    columns 2i, 2i+1 stay adjacent; oracle/mf.c: factor_front)
};

// C(m x n, ldc) -= A(m x k, lda) * B(k x n, ldb), column-major; tiles of 64 x 64 numbered
// from tile0 within one launch (tasks sorted by tile0).  C may alias A (C = A, n <= tile width)
// or B (C = B, m <= tile height): every tile reads all of its A rows / B columns before it
// stores, which the GEMM-form triangular solves use (C - (I - T^-1) C = T^-1 C).
struct GemmTask {
  const double* A;
  const double* B;
  double* C;
  int32_t m, n, k;
  int32_t lda, ldb, ldc;
  int32_t tiles_m;
  int32_t gsid = -1; // >= 0: growth check of the result (GEMM-form TRSM of front gsid's L rows)
  int64_t tile0;
};

// Fused U rows of an outer block (k_urows): one kUrowsCols-column block of the columns right of
// the block; rows [ob0, ob1) of the block solved sub-panel by sub-panel (tinv slots slot0 + u).
constexpr int kUrowsCols = 32;
struct URowTask {
  int32_t s;
  int32_t ob0, ob1;
  int32_t slot0;
  int32_t ld;      // M for L-panel columns, ns for U12 columns
  int32_t ncols;   // <= kUrowsCols
  int64_t coff;    // store offset of (row 0, first column) of the block
};

// Per-launch front lists for the blocked path: front id + first workgroup index.
struct FrontTile {
  int32_t s;
  int32_t pad;
  int64_t wg0;
};

// Extend-add task: parent front p's column tj receives cnt child columns, listed as (child,
// child column) pairs at contrib[off, off+cnt) in child order.
// Assembly task: column tj of front p.  Child contributions xtasks[off, off+cnt) in child order;
// A entries aents[aoff, aoff+acnt) as (entry id, local row), rows ascending.
// One child F22 column contributing to a parent column: the child (its nu and row map) and where
// the column's nu values are: src >= 0 -> scratch + src, src < 0 -> store + (-1 - src).
struct XContrib {
  int32_t child, pad;
  int64_t src;
};

// Device-to-device copy of n4 4-byte words (the pack / unpack steps of the multi-GPU exchanges).
struct SegDesc {
  uint64_t src, dst;
  int64_t n4;
};

struct XCol {
  int32_t p, tj;
  int64_t off;
  int32_t cnt, acnt;
  int64_t aoff;
};

// Row swaps of one or more consecutive panels (sub-panels kb0 + u*nb, swap-list slots slot0 + u,
// u < nsub) applied in order to the front columns [a, b) minus [c_lo, c_hi); 64 columns per
// workgroup, workgroups numbered from wg0 within one launch (tasks sorted by wg0).
struct SwapTask {
  int32_t s, kb0, nsub, slot0;
  int32_t a, b, c_lo, c_hi;
  int64_t wg0;
};

// Right-hand sides of a solve launch: n vectors, vector r of x at x + r*ldx and of the front
// vectors at vbuf + r*ldv.
struct Rhs {
  int32_t n;
  int64_t ldx, ldv;
};
constexpr int kMultiRhs = 16;   // right-hand sides per solve launch
#ifndef SMLU_SWEEP_WK
#define SMLU_SWEEP_WK 4
#endif
constexpr int kSweepWK = SMLU_SWEEP_WK;   // k_tri_sweep: 64-row blocks (worker waves) per work item
constexpr int kSweepXB = 64;    // k_tri_sweep: external blocks x right-hand sides per run (LDS 32 KB)
// One dense chunk of the reference's solve layout (src/SharedMemSparseLU.jl:101-243), 0-based:
// the s x s diagonal block over x[c0, c0+s) at data[tri] (column-major, ld s) and the negated
// nr x s rectangle over rows x[r0, r0+nr) at data[rect] (column-major, ld nr).
struct ChunkDesc {
  int64_t c0, s, r0, nr, tri, rect;
};

}  // namespace smlu
