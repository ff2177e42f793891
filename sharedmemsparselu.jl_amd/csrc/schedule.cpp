// schedule.cpp — the static launch schedule of the multifrontal refactorization and the solves
// (built once per plan and pivoting mode) and the device buffers it addresses.
#include "handle.hpp"

// ---------------------------------------------------------------------------------------
// Schedule construction (host, once per plan)
// ---------------------------------------------------------------------------------------
// Staging of the communication steps: device send / receive staging (largest step) and the
// pinned host staging of a host-memory transport (every peer's message side by side).
static void stage_sizes(const smlu_handle* h, int64_t& ss, int64_t& rs, int64_t& hs, int64_t& hr) {
  ss = rs = hs = hr = 0;
  for (const CommOp& op : h->comm) {
    int64_t a = 0, b = 0, sa = 0, sb = 0;
    for (size_t i = 0; i < op.peer.size(); ++i) {
      if (op.sbase[i] == 4) a = std::max(a, op.soff[i] + op.sbytes[i]);
      if (op.rbase[i] == 5) b = std::max(b, op.roff[i] + op.rbytes[i]);
      sa += op.sbytes[i];
      sb += op.rbytes[i];
    }
    if (op.type == 1 && op.bbase == 4) a = std::max(a, op.bytes);
    ss = std::max(ss, a);
    rs = std::max(rs, b);
    hs = std::max(hs, std::max(sa, op.type == 1 ? op.bytes : 0));
    hr = std::max(hr, std::max(sb, op.type == 1 ? op.bytes : 0));
  }
}

static int build_schedule(smlu_handle* h) {
  Plan& P = h->plan;
  const Tune tn = tune();
  const int64_t nsup = P.nsup;
  hipStream_t st = h->stream;
  // supernode records: fronts [0, nsup) with this rank's offsets (RankLayout); a shared front
  // (multi-GPU) keeps a front node for its solves and the row maps, plus one block node per
  // owned column block whose offsets are shifted so that the front's column c of the block sits
  // at the usual place (pivot block: L + c*M; update block: U + (c-ns)*ns, F + (c-ns)*nu)
  const RankLayout& Y = h->lay;
  h->hsn.resize(nsup);
  int64_t voff = 0;
  // Largest ns factored with full-candidate pivoting.  A diagonally dominant matrix needs no
  // row exchanges (partial pivoting keeps the diagonal and the Schur complements stay
  // dominant), so there every blocked front takes the faster diagonal-tile path (round 6: the
  // mid-size fronts too -- C2 refactor 5.42 -> 3.51 ms, 128^3 465 -> 461 ms); its growth check
  // still flags weak pivots if a refactor's new values lose dominance (the re-pivoting refactor
  // then runs).  SMLU_FULLPIV_NS overrides (dev).
  // a complex handle's pair-preserving pivots search every fully-summed row (mode 1): the
  // diagonal-tile panels have no pair rule
  const int64_t full_piv_ns = (h->pivmode == 1 || h->cpair) ? std::numeric_limits<int64_t>::max()
                              : tn.fullpiv_ns >= 0 ? tn.fullpiv_ns
                              : h->dominant ? (int64_t)0 : (int64_t)kFullPivNs;
  for (int64_t s = 0; s < nsup; ++s) {
    SNode r{};
    r.first = P.s_first[s];
    r.Loff = Y.Loff[s] >= 0 ? Y.Loff[s] : 0;
    r.Uoff = Y.Uoff[s] >= 0 ? Y.Uoff[s] : 0;
    r.Foff = Y.Foff[s];
    r.rowptr = P.s_rowptr[s];
    r.voff = voff;
    r.ns = (int32_t)P.ns(s);
    r.nu = (int32_t)P.nu(s);
    voff += P.M(s);
    r.parent = (int32_t)P.s_parent[s];
    int64_t M = P.M(s);
    if (M <= kSmallM) { r.mode = 0; r.nb = 0; }
    else if (r.ns <= full_piv_ns) { r.mode = 1; r.nb = kNbFull; }
    else { r.mode = 2; r.nb = kNbTile; }
    if (h->opts.pivot_tol <= 0) { /* no pivoting requested: tile mode never searches far */ }
    r.chbeg = (int32_t)P.ch_ptr[s];
    r.chend = (int32_t)P.ch_ptr[s + 1];
    r.level = P.s_level[s];
    r.cpair = h->cpair ? 1 : 0;
    if (h->nranks > 1 && P.dist(s)) { r.mode = 2; r.nb = kNbTile; }   // shared fronts: diagonal-tile pivoting
    h->hsn[s] = r;
  }
  h->node_front.resize(nsup);
  for (int64_t s = 0; s < nsup; ++s) h->node_front[s] = (int32_t)s;
  std::vector<int32_t> blknode(Y.blocks.size());
  std::unordered_map<int64_t, int32_t> blkmap;   // (front, block) -> index in Y.blocks
  for (size_t i = 0; i < Y.blocks.size(); ++i) {
    const RankLayout::Blk& B = Y.blocks[i];
    SNode r = h->hsn[B.s];
    const int64_t ns = r.ns, nu = r.nu, M = ns + nu;
    if (B.c0 < ns) {
      r.Loff = B.loff - B.c0 * M;
    } else {
      r.Uoff = B.loff - (B.c0 - ns) * ns;
      r.Foff = B.foff - (B.c0 - ns) * nu;
    }
    blknode[i] = (int32_t)h->hsn.size();
    blkmap[(int64_t)B.s * 1048576 + B.b] = (int32_t)i;
    h->hsn.push_back(r);
    h->node_front.push_back(B.s);
  }
  h->nnodes = (int64_t)h->hsn.size();
  // given (p,q): no pivoting on top of the caller's order -> tile mode pivots only if the
  // diagonal is exactly zero; we force diag preference by a tiny diag tolerance at launch.
  std::vector<int32_t> ilist;
  std::vector<XContrib> xt;
  std::vector<FrontTile> ft;
  std::vector<int32_t> gptr, gent;   // k_fwd_pull lists
  std::vector<GemmTask> gt;
  std::vector<SwapTask> st_tasks;
  std::vector<URowTask> ur_tasks;
  std::vector<XCol> xc;
  std::vector<int2> ae;
  // A entries grouped by front, sorted by (local column, local row)
  std::vector<int64_t> fr_ptr(nsup + 1, 0);
  std::vector<int32_t> fr_ent((size_t)P.nnzA);
  {
    for (int64_t e = 0; e < P.nnzA; ++e) ++fr_ptr[P.A_s[e] + 1];
    for (int64_t s = 0; s < nsup; ++s) fr_ptr[s + 1] += fr_ptr[s];
    std::vector<int64_t> fp(fr_ptr.begin(), fr_ptr.end() - 1);
    for (int64_t e = 0; e < P.nnzA; ++e) fr_ent[fp[P.A_s[e]]++] = (int32_t)e;
    // (only the fronts this rank assembles: its own and the shared ones of its groups)
    for (int64_t s = 0; s < nsup; ++s) {
      if (h->nranks > 1 && !(P.dist(s) ? std::binary_search(P.group[s].begin(), P.group[s].end(), h->rank)
                                       : P.owner[s] == h->rank))
        continue;
      std::sort(fr_ent.begin() + fr_ptr[s], fr_ent.begin() + fr_ptr[s + 1], [&](int32_t a, int32_t b) {
        return P.A_lj[a] != P.A_lj[b] ? P.A_lj[a] < P.A_lj[b] : P.A_li[a] < P.A_li[b];
      });
    }
  }
  double* store = h->store.p;
  double* scratch = h->scratch.p;
  h->fac.clear();
  // this rank's fronts by level (every front when nranks == 1)
  std::vector<int64_t> LP(P.nlevels + 1, 0);
  std::vector<int32_t> LS;
  std::vector<std::vector<int32_t>> dfront(P.nlevels);   // shared fronts this rank works on, per level
  std::vector<char> dlevel(P.nlevels, 0);          // a level holding any shared front (any rank)
  for (int l = 0; l < P.nlevels; ++l) {
    for (int64_t k = P.lev_ptr[l]; k < P.lev_ptr[l + 1]; ++k) {
      const int64_t s = P.lev_sup[k];
      if (h->nranks == 1) { LS.push_back((int32_t)s); continue; }
      if (!P.dist(s)) {
        if (P.owner[s] == h->rank) LS.push_back((int32_t)s);
        continue;
      }
      dlevel[l] = 1;
      if (std::binary_search(P.group[s].begin(), P.group[s].end(), h->rank)) dfront[l].push_back((int32_t)s);
    }
    LP[l + 1] = (int64_t)LS.size();
  }
  h->fac_seg.assign(1, 0);
  h->fwd_seg.assign(1, 0);
  h->bwd_seg.assign(1, 0);
  h->fac_comm.clear();
  h->fwd_comm.clear();
  h->bwd_comm.clear();
  h->comm.clear();
  // a communication step ends the current segment of `seq`
  auto add_comm = [&](std::vector<Launch>& seq, std::vector<size_t>& seg, std::vector<int>& cm, CommOp&& op) {
    seg.push_back(seq.size());
    cm.push_back((int)h->comm.size());
    h->comm.push_back(std::move(op));
  };
  const int dist_slots = h->nranks > 1 ? h->ob / 32 : 0;   // swap / tile-inverse slots of the shared front
  // where child column jc of c lives: (rank, scratch offset on that rank if it is this rank)
  auto child_col = [&](int64_t c, int64_t jc, int64_t* src) -> int32_t {
    const int64_t nuc = P.nu(c);
    if (!P.dist(c)) {
      if (src && P.owner[c] == h->rank) *src = Y.Foff[c] + jc * nuc;
      return P.owner[c];
    }
    const int64_t b = P.npblk(c) + jc / P.dob;
    const int32_t o = P.blk_owner(c, b);
    if (src && o == h->rank) {
      const RankLayout::Blk& B = Y.blocks[blkmap.at((int64_t)c * 1048576 + b)];
      *src = B.foff + (P.ns(c) + jc - B.c0) * nuc;
    }
    return o;
  };
  if (tn.ob > 0) h->ob = tn.ob;
  h->t128_min = tn.t128_min;
  h->small_k = tn.small_k;
  // MFMA 128 tile: code 131 (v3: LDS-DMA staging, kernels_gemm.hip); the F22 launches (k = ns, the
  // long-k shapes) take 135, the same tile with the next slice's barrier between its last two
  // k-quads (+3 % at k >= 2048, neutral at the k = 384 trailing shapes: tools/gemm_bench)
  const int mfma_tile = 131;
  // GEMM-form TRSM (k_tri_inv + GEMM tasks) needs the growth epilogue of the MFMA/64 tiles
  // (the 32-wide panels keep k_step_trsm: measured best)
  h->trsm_gemm = h->opts.use_mfma;
  // GEMM tasks whose A or B operand lives in the tinv buffer (allocated after the schedule)
  std::vector<std::pair<int64_t, int64_t>> tinv_patch;   // (gt index * 2 + operand B?, offset)
  h->gemm_flops = 0;
  h->gemm_launches = h->gemm128_launches = 0;
  h->gemm_bytes = 0;
  h->gemm22_flops = 0;
  h->dense_flops = P.flops;
  int64_t max_list = 1;
  // GEMM launches: 128x128 tiles when the launch has enough of them to fill the GPU,
  // otherwise 64x64 tiles (same per-element arithmetic, bitwise-identical results).
  auto add_gemm_launch = [&](std::vector<GemmTask>& cand, double fl, int step, int kind = K_GEMM,
                             const std::vector<int64_t>* tpatch = nullptr) {
    if (cand.empty()) return;
    const bool count = kind != K_TRSML;   // GEMM-form TRSM is accounted as "trsm", not GEMM
    int64_t t128 = 0;
    for (auto& g : cand) t128 += (int64_t)((g.m + 127) / 128) * ((g.n + 127) / 128);
    // GEMM-form TRSM (k = n = w <= 64: tall L-row and wide U-row strips) always on the one-shot
    // 64 x 64 tile: the 128 tile would take its generic edge body for the 64-wide strips
    // (round 5: TRSM 23.0 -> 21.3 ms per 128^3 refactor)
    int tile = t128 >= h->t128_min && !(kind == K_TRSML && h->small_k) ? 128 : 64;
    if (tile == 128) tile = h->opts.use_mfma ? mfma_tile : 64;   // use_mfma = 0: the VALU 64 tile
    if (tile == 131 && step < 0) tile = 135;
    if (tile == 64 && h->small_k) {                    // every k <= 64: one-shot K staging
      int kmax = 0;
      for (auto& g : cand) kmax = std::max(kmax, g.k);
      tile = kmax <= 64 ? 65 : h->opts.use_mfma ? 66 : 64;   // 66: the 64 tile on the matrix cores
    }
    if (step < 0 && !tpatch)   // F22: longest k first, so the launch's last tiles are short ones
      std::stable_sort(cand.begin(), cand.end(), [](const GemmTask& a, const GemmTask& b) { return a.k > b.k; });
    Launch L;
    L.kind = step < 0 ? K_GEMM22 : kind;
    L.step = step;
    L.off = (int64_t)gt.size();
    L.aux = tile;
    int64_t tiles = 0;
    const int ts = tile >= 128 ? 128 : 64;
    for (size_t i = 0; i < cand.size(); ++i) {
      GemmTask& g = cand[i];
      if (count) h->gemm_bytes += 8.0 * ((double)g.m * g.k + (double)g.k * g.n + 2.0 * g.m * g.n);
      if (tpatch && (*tpatch)[i] >= 0) tinv_patch.push_back({(int64_t)gt.size(), (*tpatch)[i]});
      g.tiles_m = (g.m + ts - 1) / ts;
      g.tile0 = tiles;
      tiles += (int64_t)g.tiles_m * ((g.n + ts - 1) / ts);
      gt.push_back(g);
    }
    L.cnt = (int64_t)cand.size();
    L.nwg = tiles;
    L.flops = fl;
    h->fac.push_back(L);
    if (!count) return;
    h->gemm_flops += fl;
    ++h->gemm_launches;
    if (tile >= 128) ++h->gemm128_launches;
    if (step < 0) h->gemm22_flops += fl;
  };
  // fronts whose triangular solves run in GEMM form (tile inverses); they also take the
  // super-block level of the three-level blocking (SB columns; OB for the others)
  auto gform = [&](int64_t s) {
    return h->trsm_gemm && h->hsn[s].nb == kNbTile;
  };
  const int64_t spf = h->ob / 32;   // swap / tile-inverse slots per front
  // fused panels (k_panel_blk<16, true>: panel + tile inverses + in-block row interchanges) for
  // the GEMM-form fronts (every 64-wide panel then belongs to one); SMLU_FUSED_PANEL=0: three launches
  // 2 (default): panel + the in-block row interchanges (no k_laswp inside the block) + the tile
  // inverses by 16 x 16 blocks on the matrix cores (no k_tri_inv); 1: without the inverses;
  // 0: three launches
  const int fuse_mode = !(h->trsm_gemm && h->ob <= 64 + 16 * 20) ? 0 : 2;
  const bool fuse_panel = fuse_mode > 0, fuse_inv = fuse_mode == 2;
  // fused U rows at the end of an outer block (k_urows) for the GEMM-form fronts; SMLU_FUSED_UROWS=0:
  // one TRSM + one update launch per sub-panel
  const bool fuse_urows = h->ob <= 384;
  // tinv operand encoding in tpatch: offset * 2 + (1 if the operand is B, 0 if A)
  auto tinv_slot_off = [](int64_t slot, bool upper) { return slot * 8192 + (upper ? 4096 : 0); };
  for (int l = 0; l < P.nlevels; ++l) {
    Launch L;
    // (shared fronts of this level, in front order on every rank)
    // shared front: the children's F22 columns move to the owners of the target columns; a
    // rank receives them into its receive area ordered by (source rank, child, column)
    std::unordered_map<int64_t, int64_t> recv_at;   // (child, column) -> scratch offset
    for (const int32_t t : dfront[l]) {
      CommOp op;
      std::vector<std::vector<std::pair<int64_t, int64_t>>> from(h->nranks);   // per source: (c, jc)
      for (int64_t e = P.ch_ptr[t]; e < P.ch_ptr[t + 1]; ++e) {
        const int64_t c = P.ch_list[e];
        const int32_t* rm = P.relmap.data() + P.s_rowptr[c];
        const int64_t nuc = P.nu(c);
        for (int64_t jc = 0; jc < nuc; ++jc) {
          const int32_t dst = P.col_owner(t, rm[jc]);
          int64_t src = -1;
          const int32_t o = child_col(c, jc, &src);
          if (o == dst) continue;
          if (o == h->rank) {            // send: pack into the staging buffer
            const int pi = op.at(dst);
            op.pack.push_back(HSeg{1, 8 * src, 4, 0, 8 * nuc});   // staging offset fixed below
            op.pack.back().db = 1000 + pi;                           // peer marker
            op.sbytes[pi] += 8 * nuc;
          } else if (dst == h->rank) {
            from[o].push_back({c, jc});
          }
        }
      }
      int64_t ro = Y.recv_off[t];
      for (int32_t o = 0; o < h->nranks; ++o) {
        if (from[o].empty()) continue;
        const int pi = op.at(o);
        op.rbase[pi] = 1;
        op.roff[pi] = 8 * ro;
        for (auto& cj : from[o]) {
          recv_at[cj.first * 1048576 + cj.second] = ro;
          ro += P.nu(cj.first);
          op.rbytes[pi] += 8 * P.nu(cj.first);
        }
      }
      // send staging offsets: per peer contiguous, in (child, column) order
      {
        std::vector<int64_t> base(op.peer.size(), 0);
        int64_t acc = 0;
        for (size_t i = 0; i < op.peer.size(); ++i) {
          op.soff[i] = acc;
          base[i] = acc;
          acc += op.sbytes[i];
        }
        for (auto& g : op.pack) {
          const int pi = g.db - 1000;
          g.db = 4;
          g.dof = base[pi];
          base[pi] += g.bytes;
        }
      }
      add_comm(h->fac, h->fac_seg, h->fac_comm, std::move(op));
    }
    // assembly: every column of this level's fronts built once (zeros, scaled A entries, the
    // children's F22 columns in child order) -- k_assemble, one wave per column
    {
      L = Launch();
      L.kind = K_EXTADD;
      L.off = (int64_t)xc.size();
      std::vector<int32_t> cnt, pos;
      auto front_columns = [&](int64_t s, const std::vector<std::pair<int64_t, int64_t>>& ranges,
                               const std::vector<int32_t>& nodes) {
        const int64_t M = P.M(s);
        cnt.assign(M + 1, 0);
        for (int64_t ci = P.ch_ptr[s]; ci < P.ch_ptr[s + 1]; ++ci) {
          const int64_t c = P.ch_list[ci];
          const int32_t* rm = P.relmap.data() + h->hsn[c].rowptr;
          for (int64_t jc = 0; jc < P.nu(c); ++jc) ++cnt[rm[jc] + 1];
        }
        for (int64_t tj = 0; tj < M; ++tj) cnt[tj + 1] += cnt[tj];
        const int64_t base = (int64_t)xt.size();
        xt.resize(base + cnt[M]);
        pos.assign(cnt.begin(), cnt.end() - 1);
        for (int64_t ci = P.ch_ptr[s]; ci < P.ch_ptr[s + 1]; ++ci) {
          const int64_t c = P.ch_list[ci];
          const int32_t* rm = P.relmap.data() + h->hsn[c].rowptr;
          for (int64_t jc = 0; jc < P.nu(c); ++jc) {
            int64_t src = -1;
            if (h->nranks == 1) src = h->hsn[c].Foff + jc * P.nu(c);
            else if (P.col_owner(s, rm[jc]) == h->rank) {
              if (child_col(c, jc, &src) != h->rank) src = recv_at.at(c * 1048576 + jc);
            }
            xt[base + pos[rm[jc]]++] = XContrib{(int32_t)c, 0, src};
          }
        }
        // A entries of this front by (column, row); one task per column of the given ranges
        int64_t ea = fr_ptr[s];
        const int64_t eb = fr_ptr[s + 1];
        for (size_t ri = 0; ri < ranges.size(); ++ri)
          for (int64_t tj = ranges[ri].first; tj < ranges[ri].second; ++tj) {
            while (ea < eb && P.A_lj[fr_ent[ea]] < tj) ++ea;
            const int64_t a0 = (int64_t)ae.size();
            while (ea < eb && P.A_lj[fr_ent[ea]] == tj) {
              ae.push_back(make_int2(fr_ent[ea], P.A_li[fr_ent[ea]]));
              ++ea;
            }
            xc.push_back(XCol{nodes[ri], (int32_t)tj, base + cnt[tj], cnt[tj + 1] - cnt[tj],
                              (int32_t)((int64_t)ae.size() - a0), a0});
          }
      };
      for (int64_t k = LP[l]; k < LP[l + 1]; ++k) {   // small fronts assemble inside k_front_small
        const int64_t s = LS[k];
        if (h->hsn[s].mode != 0) front_columns(s, {{0, P.M(s)}}, {(int32_t)s});
      }
      for (const int32_t t : dfront[l]) {   // the shared front: this rank's column blocks
        std::vector<std::pair<int64_t, int64_t>> ranges;
        std::vector<int32_t> nodes;
        for (size_t i = 0; i < Y.blocks.size(); ++i)
          if (Y.blocks[i].s == t) {
            ranges.push_back({Y.blocks[i].c0, Y.blocks[i].c1});
            nodes.push_back(blknode[i]);
          }
        front_columns(t, ranges, nodes);
      }
      L.cnt = (int64_t)xc.size() - L.off;
      if (L.cnt > 0) h->fac.push_back(L);
    }
    // small fronts (assembly fused into the factorization), launched per size class so that
    // small fronts get small LDS (occupancy); ilist: (front, first A entry, A entry count), the
    // front's A entries as (entry, local column << 16 | local row)
    {
      const int64_t cls[6] = {16, 32, 48, 64, 96, kSmallM};
      for (int c = 0; c < 6; ++c) {
        L = Launch();
        L.kind = K_FRONT_LDS;
        L.off = (int64_t)ilist.size();
        int64_t Mmax = 0;
        for (int64_t k = LP[l]; k < LP[l + 1]; ++k) {
          int64_t s = LS[k];
          if (h->hsn[s].mode != 0) continue;
          int64_t M = P.M(s);
          if (M > cls[c] || (c > 0 && M <= cls[c - 1])) continue;
          ilist.push_back((int32_t)s);
          ilist.push_back((int32_t)ae.size());
          ilist.push_back((int32_t)(fr_ptr[s + 1] - fr_ptr[s]));
          for (int64_t e = fr_ptr[s]; e < fr_ptr[s + 1]; ++e) {
            const int32_t id = fr_ent[e];
            ae.push_back(make_int2(id, (int32_t)((P.A_lj[id] << 16) | P.A_li[id])));
          }
          Mmax = std::max(Mmax, M);
        }
        L.cnt = ((int64_t)ilist.size() - L.off) / 3;
        L.aux = Mmax;
        // overlap group: the size classes of one level run on two streams (factor.cpp).  That is
        // race-free only because the scratch plan (plan.cpp: one F22 block per level, live until
        // the parents' level) keeps every F22 a front of this level writes disjoint from every
        // other one and from the children's F22 the level reads -- checked below.  (Round 6: the
        // level's blocked fronts on a third stream next to them, C2 3.51 -> 4.25 ms: not kept.)
        L.aux2 = l + 1;
        if (L.cnt > 0) h->fac.push_back(L);
      }
      std::vector<std::pair<int64_t, int64_t>> wr, rd;   // F22 ranges written / read by the level
      for (int64_t k = LP[l]; k < LP[l + 1]; ++k) {
        const int64_t s = LS[k];
        if (h->hsn[s].mode != 0) continue;
        const int64_t nu = P.nu(s);
        if (nu > 0 && h->hsn[s].Foff >= 0) wr.push_back({h->hsn[s].Foff, h->hsn[s].Foff + nu * nu});
        for (int64_t e = P.ch_ptr[s]; e < P.ch_ptr[s + 1]; ++e) {
          const int64_t c = P.ch_list[e], nuc = P.nu(c);
          if (nuc > 0 && h->hsn[c].Foff >= 0) rd.push_back({h->hsn[c].Foff, h->hsn[c].Foff + nuc * nuc});
        }
      }
      std::sort(wr.begin(), wr.end());
      for (size_t i = 1; i < wr.size(); ++i)
        if (wr[i].first < wr[i - 1].second) return fail(h, SMLU_ERR_STATE, "internal: overlapping F22 blocks in one level");
      for (const auto& r : rd) {   // a read range must not meet any written range
        auto it = std::upper_bound(wr.begin(), wr.end(), std::make_pair(r.second, (int64_t)-1));
        if (it != wr.begin() && std::prev(it)->second > r.first)
          return fail(h, SMLU_ERR_STATE, "internal: a level's F22 block overlaps a child's F22 it reads");
      }
    }
    // blocked fronts
    std::vector<int64_t> big;
    std::unordered_map<int64_t, int64_t> bidx;   // front -> index in big (swap-list slots)
    int64_t maxsteps = 0;
    for (int64_t k = LP[l]; k < LP[l + 1]; ++k) {
      int64_t s = LS[k];
      const SNode& r = h->hsn[s];
      if (r.mode == 0) continue;
      bidx[s] = (int64_t)big.size();
      big.push_back(s);
      maxsteps = std::max<int64_t>(maxsteps, (r.ns + r.nb - 1) / r.nb);
    }
    max_list = std::max<int64_t>(max_list, dist_slots + (int64_t)big.size() * spf);
    // swap-list slot of sub-panel u of a front's current outer block
    auto slot_of = [&](int64_t s, int64_t u) { return dist_slots + bidx[s] * spf + u; };
    for (int64_t t = 0; t < maxsteps; ++t) {
      std::vector<int64_t> act;
      for (auto s : big) {
        const SNode& r = h->hsn[s];
        if (t * r.nb < r.ns) act.push_back(s);
      }
      if (act.empty()) continue;
      // panel launch classes by register-kernel shape: (W=64, 1 wave), (W=32, 1/2/4/8 waves)
      auto pclass = [&](int64_t s) {
        const SNode& r = h->hsn[s];
        int64_t kb = t * r.nb, w = std::min<int64_t>(r.nb, r.ns - kb);
        int64_t R = r.mode == 1 ? r.ns - kb : w;
        if (r.nb > 32) return 0;
        return R <= 64 ? 1 : R <= 128 ? 2 : R <= 256 ? 3 : R <= 512 ? 4 : 5;
      };
      std::stable_sort(act.begin(), act.end(), [&](int64_t a, int64_t b) { return pclass(a) < pclass(b); });
      {
        size_t pos = 0;
        for (int c = 0; c < 6 && pos < act.size(); ++c) {
          L = Launch();
          L.kind = K_PANEL;
          L.step = (int)t;
          L.off = (int64_t)ilist.size();
          int64_t rmax = 1, wmax = 1, cnt = 0;
          while (pos < act.size() && pclass(act[pos]) == c) {
            const SNode& r = h->hsn[act[pos]];
            int64_t kb = t * r.nb, w = std::min<int64_t>(r.nb, r.ns - kb);
            rmax = std::max(rmax, r.mode == 1 ? r.ns - kb : w);
            wmax = std::max<int64_t>(wmax, r.nb);
            ilist.push_back((int32_t)act[pos]);
            ilist.push_back((int32_t)slot_of(act[pos], t % (h->ob / r.nb)));
            ++pos;
            ++cnt;
          }
          L.cnt = cnt;
          L.aux = 0;
          L.nwg = rmax;
          L.aux2 = wmax;
          L.cnt2 = c == 0 ? fuse_mode : 0;   // 64-wide panels of GEMM-form fronts: fused tail
          if (L.cnt > 0) h->fac.push_back(L);
        }
        if (pos != act.size()) return fail(h, SMLU_ERR_ARG, "internal: panel classes");
      }
      // inverses of the diagonal tiles of the GEMM-form fronts (I - L_kk^-1, I - U_kk^-1)
      {
        L = Launch();
        L.kind = K_TRIINV;
        L.step = (int)t;
        L.off = (int64_t)ilist.size();
        for (auto s : act) {
          if (!gform(s) || fuse_inv) continue;   // fused into the panel launch
          ilist.push_back((int32_t)s);
          ilist.push_back((int32_t)slot_of(s, t % (h->ob / h->hsn[s].nb)));
        }
        L.cnt = ((int64_t)ilist.size() - L.off) / 2;
        if (L.cnt > 0) h->fac.push_back(L);
      }
      // row swaps inside the outer block (the other columns get them at the end of the block)
      {
        L = Launch();
        L.kind = K_LASWP;
        L.step = (int)t;
        L.off = (int64_t)st_tasks.size();
        int64_t wg = 0;
        for (auto s : act) {
          const SNode& r = h->hsn[s];
          int64_t kb = t * r.nb, w = std::min<int64_t>(r.nb, r.ns - kb);
          int64_t ostart = (kb / h->ob) * h->ob, oend = std::min<int64_t>(r.ns, ostart + h->ob);
          int64_t ncol = oend - ostart - w;
          if (ncol <= 0 || (fuse_panel && gform(s))) continue;   // fused panels swap these rows themselves
          st_tasks.push_back(SwapTask{(int32_t)s, (int32_t)kb, 1, (int32_t)slot_of(s, t % (h->ob / r.nb)),
                                      (int32_t)ostart, (int32_t)oend, (int32_t)kb, (int32_t)(kb + w), wg});
          wg += (ncol + 63) / 64;
        }
        L.cnt = (int64_t)st_tasks.size() - L.off;
        L.nwg = wg;
        if (wg > 0) h->fac.push_back(L);
      }
      {
        Launch T;
        T.kind = K_STEPTRSM;
        T.step = (int)t;
        T.off = (int64_t)ft.size();
        int64_t wgU = 0, W = 32, ntri = 0;
        for (auto s : act) {
          if (gform(s)) continue;
          ++ntri;
          const SNode& r = h->hsn[s];
          int64_t kb = t * r.nb, w = std::min<int64_t>(r.nb, r.ns - kb);
          int64_t ostart = (kb / h->ob) * h->ob, oend = std::min<int64_t>(r.ns, ostart + h->ob);
          ft.push_back(FrontTile{(int32_t)s, (int32_t)kb, wgU});
          wgU += (oend - kb - w + 255) / 256;
          W = std::max<int64_t>(W, w);
        }
        T.cnt = ntri;
        T.nwg = wgU;
        T.off2 = (int64_t)ft.size();
        int64_t wgL = 0;
        for (auto s : act) {
          if (gform(s)) continue;
          const SNode& r = h->hsn[s];
          int64_t M = (int64_t)r.ns + r.nu, kb = t * r.nb, w = std::min<int64_t>(r.nb, r.ns - kb);
          int64_t R = r.mode == 1 ? r.ns - kb : w;
          ft.push_back(FrontTile{(int32_t)s, (int32_t)kb, wgL});
          wgL += (M - kb - R + 255) / 256;
        }
        T.cnt2 = ntri;
        T.nwg2 = wgL;
        T.aux = W;
        if (wgU + wgL > 0) h->fac.push_back(T);
      }
      // GEMM-form step TRSM of the blocked fronts, in place (R = rows the panel finished:
      // w for diagonal-tile panels, every fully-summed row for full-candidate panels):
      //   U rows [kb, kb+w) x columns [kb+w, oend):  C - (I - L_kk^-1) C = L_kk^-1 C
      //   L rows [kb+R, M) x columns [kb, kb+w):     C - C (I - U_kk^-1) = C U_kk^-1 (+ growth)
      {
        std::vector<GemmTask> cand;
        std::vector<int64_t> tp;
        for (auto s : act) {
          if (!gform(s)) continue;
          const SNode& r = h->hsn[s];
          int64_t M = (int64_t)r.ns + r.nu, kb = t * r.nb, w = std::min<int64_t>(r.nb, r.ns - kb);
          int64_t ostart = (kb / h->ob) * h->ob, oend = std::min<int64_t>(r.ns, ostart + h->ob);
          const int64_t slot = slot_of(s, t % (h->ob / r.nb));
          if (oend - kb - w > 0) {
            GemmTask g{};
            g.B = g.C = store + r.Loff + (kb + w) * M + kb;
            g.m = (int)w; g.n = (int)(oend - kb - w); g.k = (int)w;
            g.lda = 64; g.ldb = (int)M; g.ldc = (int)M;
            cand.push_back(g);
            tp.push_back(tinv_slot_off(slot, false) * 2);
          }
          const int64_t R = r.mode == 1 ? r.ns - kb : w;   // rows the panel already finished
          if (M - kb - R > 0) {
            GemmTask g{};
            g.A = g.C = store + r.Loff + kb * M + kb + R;
            g.m = (int)(M - kb - R); g.n = (int)w; g.k = (int)w;
            g.lda = (int)M; g.ldb = 64; g.ldc = (int)M;
            g.gsid = (int32_t)s;
            cand.push_back(g);
            tp.push_back(tinv_slot_off(slot, true) * 2 + 1);
          }
        }
        add_gemm_launch(cand, 0.0, (int)t, K_TRSML, &tp);
      }
      // inner trailing update: rows [kb+w, M) x columns [kb+w, oend) of the outer block
      {
        std::vector<GemmTask> cand;
        double fl = 0;
        for (auto s : act) {
          const SNode& r = h->hsn[s];
          int64_t M = (int64_t)r.ns + r.nu, kb = t * r.nb, w = std::min<int64_t>(r.nb, r.ns - kb);
          int64_t ostart = (kb / h->ob) * h->ob, oend = std::min<int64_t>(r.ns, ostart + h->ob);
          int64_t m1 = M - kb - w, n1 = oend - kb - w;
          if (m1 > 0 && n1 > 0) {
            GemmTask g{};
            g.A = store + r.Loff + kb * M + kb + w;
            g.B = store + r.Loff + (kb + w) * M + kb;
            g.C = store + r.Loff + (kb + w) * M + kb + w;
            g.m = (int)m1; g.n = (int)n1; g.k = (int)w;
            g.lda = (int)M; g.ldb = (int)M; g.ldc = (int)M;
            cand.push_back(g);
            fl += 2.0 * m1 * n1 * w;
          }
        }
        add_gemm_launch(cand, fl, (int)t);
      }
      // end of an outer block [ostart, oend): deferred row swaps on the columns outside it, the
      // U rows of the block right of it, and the trailing update with k = oend - ostart
      std::vector<int64_t> fin_all;
      for (auto s : act) {
        const SNode& r = h->hsn[s];
        int64_t kb = t * r.nb, w = std::min<int64_t>(r.nb, r.ns - kb);
        int64_t ostart = (kb / h->ob) * h->ob, oend = std::min<int64_t>(r.ns, ostart + h->ob);
        if (kb + w == oend) fin_all.push_back(s);
      }
      if (fin_all.empty()) continue;
      {
        L = Launch();
        L.kind = K_LASWP;
        L.step = (int)t;
        L.off = (int64_t)st_tasks.size();
        int64_t wg = 0;
        for (auto s : fin_all) {
          const SNode& r = h->hsn[s];
          int64_t M = (int64_t)r.ns + r.nu, kb = t * r.nb;
          int64_t ostart = (kb / h->ob) * h->ob, oend = std::min<int64_t>(r.ns, ostart + h->ob);
          int64_t ncol = M - (oend - ostart);
          if (ncol <= 0) continue;
          st_tasks.push_back(SwapTask{(int32_t)s, (int32_t)ostart, (int32_t)((oend - ostart + r.nb - 1) / r.nb),
                                      (int32_t)slot_of(s, (ostart % h->ob) / r.nb), 0, (int32_t)M, (int32_t)ostart,
                                      (int32_t)oend, wg});
          wg += (ncol + 63) / 64;
        }
        L.cnt = (int64_t)st_tasks.size() - L.off;
        L.nwg = wg;
        if (wg > 0) h->fac.push_back(L);
      }
      // End of an outer block: its U rows on every column right of it (sub-panel by sub-panel,
      // k_urows or GEMM-form TRSM), then the trailing update with k = OB width
      struct URows {
        int64_t s, ob0, ob1, c0, c1;   // OB rows [ob0, ob1); L-panel columns [c0, c1); + U12 if u12
        bool u12;
      };
      // TRSM of the U rows of a set of OBs (one per front), sub-panel by sub-panel: L_uu^-1 C in
      // place on the given columns, then the rows below the sub-panel inside the OB
      auto urows = [&](const std::vector<URows>& all_items) {
        // GEMM-form fronts: one fused k_urows launch (every column block runs the whole
        // sub-panel sequence); the others keep one launch pair per sub-panel
        std::vector<URows> items;
        {
          L = Launch();
          L.kind = K_UROWS;
          L.step = (int)t;
          L.off = (int64_t)ur_tasks.size();
          for (auto& it : all_items) {
            const SNode& r = h->hsn[it.s];
            if (!(fuse_urows && gform(it.s))) {
              items.push_back(it);
              continue;
            }
            const int64_t M = (int64_t)r.ns + r.nu;
            const int32_t slot0 = (int32_t)slot_of(it.s, (it.ob0 % h->ob) / r.nb);
            for (int64_t c = it.c0; c < it.c1; c += kUrowsCols)
              ur_tasks.push_back(URowTask{(int32_t)it.s, (int32_t)it.ob0, (int32_t)it.ob1, slot0, (int32_t)M,
                                          (int32_t)std::min<int64_t>(kUrowsCols, it.c1 - c), r.Loff + c * M});
            if (it.u12)
              for (int64_t c = 0; c < r.nu; c += kUrowsCols)
                ur_tasks.push_back(URowTask{(int32_t)it.s, (int32_t)it.ob0, (int32_t)it.ob1, slot0, r.ns,
                                            (int32_t)std::min<int64_t>(kUrowsCols, r.nu - c), r.Uoff + c * r.ns});
          }
          L.cnt = (int64_t)ur_tasks.size() - L.off;
          if (L.cnt > 0) h->fac.push_back(L);
        }
        int64_t nsub = 0;
        for (auto& it : items) nsub = std::max<int64_t>(nsub, (it.ob1 - it.ob0 + h->hsn[it.s].nb - 1) / h->hsn[it.s].nb);
        for (int64_t u = 0; u < nsub; ++u) {
          L = Launch();
          L.kind = K_TRSMU;
          L.step = (int)t;
          L.aux = 1;   // outer mode
          L.off = (int64_t)ft.size();
          int64_t wg = 0, cnt = 0;
          std::vector<GemmTask> cand, ctri;
          std::vector<int64_t> tp;
          double fl = 0;
          for (auto& it : items) {
            const int64_t s = it.s;
            const SNode& r = h->hsn[s];
            const int64_t M = (int64_t)r.ns + r.nu;
            const int64_t kbu = it.ob0 + u * r.nb;
            if (kbu >= it.ob1) continue;
            const int64_t wu = std::min<int64_t>(r.nb, it.ob1 - kbu);
            const int64_t n1 = it.c1 - it.c0;
            if (gform(s)) {   // U rows [kbu, kbu+wu) on the columns: L_uu^-1 C, in place
              const int64_t off = tinv_slot_off(slot_of(s, (kbu % h->ob) / r.nb), false) * 2;
              if (n1 > 0) {
                GemmTask g{};
                g.B = g.C = store + r.Loff + it.c0 * M + kbu;
                g.m = (int)wu; g.n = (int)n1; g.k = (int)wu;
                g.lda = 64; g.ldb = (int)M; g.ldc = (int)M;
                ctri.push_back(g);
                tp.push_back(off);
              }
              if (it.u12 && r.nu > 0) {
                GemmTask g{};
                g.B = g.C = store + r.Uoff + kbu;
                g.m = (int)wu; g.n = r.nu; g.k = (int)wu;
                g.lda = 64; g.ldb = r.ns; g.ldc = r.ns;
                ctri.push_back(g);
                tp.push_back(off);
              }
            } else {          // k_trsm_u: columns [oend, M) of the plain two-level scheme
              ft.push_back(FrontTile{(int32_t)s, (int32_t)kbu, wg});
              wg += (M - it.c0 + 255) / 256;
              ++cnt;
            }
            // rows below the sub-panel inside the OB: [kbu+wu, ob1) x the columns
            const int64_t m = it.ob1 - kbu - wu;
            if (m > 0) {
              if (n1 > 0) {
                GemmTask g{};
                g.A = store + r.Loff + kbu * M + kbu + wu;
                g.B = store + r.Loff + it.c0 * M + kbu;
                g.C = store + r.Loff + it.c0 * M + kbu + wu;
                g.m = (int)m; g.n = (int)n1; g.k = (int)wu;
                g.lda = (int)M; g.ldb = (int)M; g.ldc = (int)M;
                cand.push_back(g);
                fl += 2.0 * m * n1 * wu;
              }
              if (it.u12 && r.nu > 0) {
                GemmTask g{};
                g.A = store + r.Loff + kbu * M + kbu + wu;
                g.B = store + r.Uoff + kbu;
                g.C = store + r.Uoff + kbu + wu;
                g.m = (int)m; g.n = r.nu; g.k = (int)wu;
                g.lda = (int)M; g.ldb = r.ns; g.ldc = r.ns;
                cand.push_back(g);
                fl += 2.0 * m * (double)r.nu * wu;
              }
            }
          }
          L.cnt = cnt;
          L.nwg = wg;
          if (wg > 0) h->fac.push_back(L);
          add_gemm_launch(ctri, 0.0, (int)t, K_TRSML, &tp);
          add_gemm_launch(cand, fl, (int)t, K_GEMMU);
        }
      };
      // C(rows [r0, r1) x L-panel columns [c0, c1) (+ U12 when u12)) -= L(rows, [k0, k1)) U([k0, k1), cols)
      auto rank_update = [&](int64_t s, int64_t r0, int64_t r1, int64_t c0, int64_t c1, bool u12, int64_t k0,
                             int64_t k1, std::vector<GemmTask>& cand, double& fl) {
        const SNode& r = h->hsn[s];
        const int64_t M = (int64_t)r.ns + r.nu, kk = k1 - k0;
        if (r1 > r0 && c1 > c0 && kk > 0) {
          GemmTask g{};
          g.A = store + r.Loff + k0 * M + r0;
          g.B = store + r.Loff + c0 * M + k0;
          g.C = store + r.Loff + c0 * M + r0;
          g.m = (int)(r1 - r0); g.n = (int)(c1 - c0); g.k = (int)kk;
          g.lda = (int)M; g.ldb = (int)M; g.ldc = (int)M;
          cand.push_back(g);
          fl += 2.0 * (double)(r1 - r0) * (double)(c1 - c0) * kk;
        }
        const int64_t ru1 = std::min<int64_t>(r1, r.ns);   // U12 rows live above ns
        if (u12 && r.nu > 0 && ru1 > r0 && kk > 0) {
          GemmTask g{};
          g.A = store + r.Loff + k0 * M + r0;
          g.B = store + r.Uoff + k0;
          g.C = store + r.Uoff + r0;
          g.m = (int)(ru1 - r0); g.n = r.nu; g.k = (int)kk;
          g.lda = (int)M; g.ldb = r.ns; g.ldc = r.ns;
          cand.push_back(g);
          fl += 2.0 * (double)(ru1 - r0) * (double)r.nu * kk;
        }
      };
      std::vector<URows> items;
      std::vector<GemmTask> c1;
      double fl1 = 0;
      for (auto s : fin_all) {
        const SNode& r = h->hsn[s];
        const int64_t kb = t * r.nb, M = (int64_t)r.ns + r.nu;
        const int64_t ostart = (kb / h->ob) * h->ob, oend = std::min<int64_t>(r.ns, ostart + h->ob);
        if (oend == M) continue;   // nothing right of the block
        items.push_back(URows{s, ostart, oend, oend, r.ns, true});
        rank_update(s, oend, M, oend, r.ns, false, ostart, oend, c1, fl1);
        rank_update(s, oend, r.ns, oend, oend, true, ostart, oend, c1, fl1);   // U12 rows only
      }
      urows(items);
      add_gemm_launch(c1, fl1, (int)t, K_GEMMO);
    }
    // F22 -= L21 * U12 for the blocked fronts of this level
    {
      std::vector<GemmTask> cand;
      double fl = 0;
      for (auto s : big) {
        const SNode& r = h->hsn[s];
        if (r.nu == 0) continue;
        int64_t M = (int64_t)r.ns + r.nu;
        GemmTask g{};
        g.A = store + r.Loff + r.ns;
        g.B = store + r.Uoff;
        g.C = scratch + r.Foff;
        g.m = r.nu; g.n = r.nu; g.k = r.ns;
        g.lda = (int)M; g.ldb = r.ns; g.ldc = r.nu;
        cand.push_back(g);
        fl += 2.0 * r.nu * (double)r.nu * r.ns;
      }
      add_gemm_launch(cand, fl, -1);
    }
    // the shared front of this level (multi-GPU): for each pivot block, its owner runs the inner
    // steps (64-column panels with diagonal-tile pivoting, tile inverses, in-block swaps, GEMM-form
    // triangular solves, in-block updates) on its copy, broadcasts the factored block (L rows
    // [ob, M), tile inverses, swap lists, rowperm) to the group, and every member applies it to
    // the column blocks it owns: deferred swaps, U rows (GEMM-form TRSM per sub-panel), the rows
    // below each sub-panel, and the trailing update (k = block width) down to the F22 rows
    for (const int32_t t : dfront[l]) {
      const SNode& fr = h->hsn[t];
      const int64_t ns = fr.ns, nu = fr.nu, M = ns + nu;
      const int64_t np = P.npblk(t);
      std::vector<size_t> mine;
      for (size_t i = 0; i < Y.blocks.size(); ++i)
        if (Y.blocks[i].s == t) mine.push_back(i);
      // look-ahead (depth 1, SMLU_DIST_LOOKAHEAD=1): the owner of pivot block b+1 applies block
      // b to block b+1 first, factors and broadcasts b+1, and only then applies b to its other
      // blocks (`pending`).  Off by default: the broadcast is a rendezvous (receivers post it
      // after their own trailing updates), so the deferred work only loads the next owner --
      // the schedule model projects 3.0x instead of 4.3x at 256^3 / 8 ranks with it on
      constexpr bool dist_lookahead = false;
      std::vector<Launch> pending;
      for (int64_t b = 0; b < np; ++b) {
        const int64_t ob = P.blk_c0(t, b), oe = P.blk_c1(t, b), w = oe - ob;
        const int64_t nsub = (w + 63) / 64;
        const int32_t o = P.blk_owner(t, b);
        const bool own = o == h->rank;
        int32_t bn = -1;
        double* Lb = nullptr;
        if (own) {
          bn = blknode[blkmap.at((int64_t)t * 1048576 + b)];
          Lb = store + h->hsn[bn].Loff;
          for (int64_t kb = ob; kb < oe; kb += 64) {
            const int64_t wk = std::min<int64_t>(64, oe - kb);
            const int step = (int)(kb / 64);
            const int32_t u = (int32_t)((kb - ob) / 64);
            Launch Q;
            Q.kind = K_PANEL;
            Q.step = step;
            Q.off = (int64_t)ilist.size();
            ilist.push_back(bn);
            ilist.push_back(u);
            Q.cnt = 1;
            Q.nwg = wk;
            Q.aux2 = 64;
            h->fac.push_back(Q);
            Q = Launch();
            Q.kind = K_TRIINV;
            Q.step = step;
            Q.off = (int64_t)ilist.size();
            ilist.push_back(bn);
            ilist.push_back(u);
            Q.cnt = 1;
            h->fac.push_back(Q);
            if (oe - ob - wk > 0) {
              Q = Launch();
              Q.kind = K_LASWP;
              Q.step = step;
              Q.off = (int64_t)st_tasks.size();
              st_tasks.push_back(SwapTask{bn, (int32_t)kb, 1, u, (int32_t)ob, (int32_t)oe, (int32_t)kb,
                                          (int32_t)(kb + wk), 0});
              Q.cnt = 1;
              Q.nwg = (oe - ob - wk + 63) / 64;
              h->fac.push_back(Q);
            }
            std::vector<GemmTask> cand;
            std::vector<int64_t> tp;
            if (oe - kb - wk > 0) {
              GemmTask g{};
              g.B = g.C = Lb + (kb + wk) * M + kb;
              g.m = (int)wk; g.n = (int)(oe - kb - wk); g.k = (int)wk;
              g.lda = 64; g.ldb = (int)M; g.ldc = (int)M;
              cand.push_back(g);
              tp.push_back(tinv_slot_off(u, false) * 2);
            }
            if (M - kb - wk > 0) {
              GemmTask g{};
              g.A = g.C = Lb + kb * M + kb + wk;
              g.m = (int)(M - kb - wk); g.n = (int)wk; g.k = (int)wk;
              g.lda = (int)M; g.ldb = 64; g.ldc = (int)M;
              g.gsid = bn;
              cand.push_back(g);
              tp.push_back(tinv_slot_off(u, true) * 2 + 1);
            }
            add_gemm_launch(cand, 0.0, step, K_TRSML, &tp);
            if (M - kb - wk > 0 && oe - kb - wk > 0) {
              GemmTask g{};
              g.A = Lb + kb * M + kb + wk;
              g.B = Lb + (kb + wk) * M + kb;
              g.C = Lb + (kb + wk) * M + kb + wk;
              g.m = (int)(M - kb - wk); g.n = (int)(oe - kb - wk); g.k = (int)wk;
              g.lda = (int)M; g.ldb = (int)M; g.ldc = (int)M;
              std::vector<GemmTask> c1{g};
              add_gemm_launch(c1, 2.0 * g.m * (double)g.n * wk, step);
            }
          }
        }
        // broadcast: [L rows [ob, M) x w, ld M-ob | tile inverses | swap lists | rowperm]
        const int64_t lbytes = 8 * (M - ob) * w, tbytes = 8 * nsub * 8192;
        const int64_t swbytes = 4 * nsub * kSwapStride, rpbytes = 4 * w;
        {
          CommOp op;
          op.type = 1;
          op.root = o;
          op.grp = P.group[t];
          op.bytes = lbytes + tbytes + swbytes + rpbytes;
          if (own) {
            op.bbase = 4;
            for (int64_t c = ob; c < oe; ++c)
              op.pack.push_back(HSeg{0, 8 * (h->hsn[bn].Loff + c * M + ob), 4, 8 * (c - ob) * (M - ob), 8 * (M - ob)});
            op.pack.push_back(HSeg{7, 0, 4, lbytes, tbytes});
            op.pack.push_back(HSeg{8, 0, 4, lbytes + tbytes, swbytes});
            op.pack.push_back(HSeg{9, 4 * (fr.first + ob), 4, lbytes + tbytes + swbytes, rpbytes});
          } else {
            op.bbase = 6;
            op.unpack.push_back(HSeg{6, lbytes + tbytes, 8, 0, swbytes});
            op.unpack.push_back(HSeg{6, lbytes + tbytes + swbytes, 9, 4 * (fr.first + ob), rpbytes});
          }
          add_comm(h->fac, h->fac_seg, h->fac_comm, std::move(op));
        }
        for (auto& q : pending) h->fac.push_back(q);   // the previous block's deferred updates
        pending.clear();
        const double* bc = h->bcbuf.p;
        const int64_t ldL = own ? M : M - ob;
        auto Lsrc = [&](int64_t row, int64_t col) -> const double* {
          return own ? Lb + col * M + row : bc + (col - ob) * (M - ob) + (row - ob);
        };
        // deferred row swaps on this rank's other blocks (left and right)
        {
          Launch Q;
          Q.kind = K_LASWP;
          Q.off = (int64_t)st_tasks.size();
          int64_t wg = 0;
          for (size_t i : mine) {
            const RankLayout::Blk& T = Y.blocks[i];
            if (T.b == b) continue;
            st_tasks.push_back(SwapTask{blknode[i], (int32_t)ob, (int32_t)nsub, 0, (int32_t)T.c0, (int32_t)T.c1,
                                        (int32_t)T.c1, (int32_t)T.c1, wg});
            wg += (T.c1 - T.c0 + 63) / 64;
          }
          Q.cnt = (int64_t)st_tasks.size() - Q.off;
          Q.nwg = wg;
          if (wg > 0) h->fac.push_back(Q);
        }
        // target blocks right of this one: (node, columns, pivot block?) and their row pointers
        struct Tgt { int32_t node; int64_t c0, c1; bool piv; };
        std::vector<Tgt> right_all, right;
        for (size_t i : mine) {
          const RankLayout::Blk& T = Y.blocks[i];
          if (T.c0 >= oe) right_all.push_back({blknode[i], T.c0, T.c1, T.c0 < ns});
        }
        // this rank owns pivot block b+1 (look-ahead): block b+1 first, the rest deferred
        const bool ahead = dist_lookahead && b + 1 < np && P.blk_owner(t, b + 1) == h->rank;
        for (int pass = 0; pass < 2; ++pass) {
        if (!ahead && pass == 1) break;
        right.clear();
        for (const Tgt& T : right_all)
          if (!ahead || (pass == 0) == (T.c0 == P.blk_c0(t, b + 1))) right.push_back(T);
        if (right.empty()) continue;
        std::vector<Launch> saved;
        if (ahead && pass == 1) saved.swap(h->fac);   // emit the deferred part into `pending`
        auto trow = [&](const Tgt& T, int64_t row) -> double* {   // rows < ns of the target's first column
          const SNode& q = h->hsn[T.node];
          return T.piv ? store + q.Loff + T.c0 * M + row : store + q.Uoff + (T.c0 - ns) * ns + row;
        };
        for (int64_t u = 0; u < nsub; ++u) {
          const int64_t kbu = ob + 64 * u, wu = std::min<int64_t>(64, oe - kbu);
          std::vector<GemmTask> ctri, cand;
          std::vector<int64_t> tp;
          double fl = 0;
          for (const Tgt& T : right) {
            const int ldt = (int)(T.piv ? M : ns);
            GemmTask g{};
            g.B = g.C = trow(T, kbu);
            g.m = (int)wu; g.n = (int)(T.c1 - T.c0); g.k = (int)wu;
            g.lda = 64; g.ldb = ldt; g.ldc = ldt;
            if (own) tp.push_back(tinv_slot_off(u, false) * 2);
            else { g.A = bc + (M - ob) * w + u * 8192; tp.push_back(-1); }
            ctri.push_back(g);
            const int64_t m = oe - kbu - wu;
            if (m > 0) {
              GemmTask q{};
              q.A = Lsrc(kbu + wu, kbu);
              q.B = trow(T, kbu);
              q.C = trow(T, kbu + wu);
              q.m = (int)m; q.n = (int)(T.c1 - T.c0); q.k = (int)wu;
              q.lda = (int)ldL; q.ldb = ldt; q.ldc = ldt;
              cand.push_back(q);
              fl += 2.0 * m * (double)(T.c1 - T.c0) * wu;
            }
          }
          add_gemm_launch(ctri, 0.0, (int)(kbu / 64), K_TRSML, &tp);
          add_gemm_launch(cand, fl, (int)(kbu / 64), K_GEMMU);
        }
        {
          std::vector<GemmTask> cand;
          double fl = 0;
          for (const Tgt& T : right) {
            const int64_t nc = T.c1 - T.c0;
            if (T.piv) {
              if (M - oe <= 0) continue;
              GemmTask g{};
              g.A = Lsrc(oe, ob);
              g.B = trow(T, ob);
              g.C = trow(T, oe);
              g.m = (int)(M - oe); g.n = (int)nc; g.k = (int)w;
              g.lda = (int)ldL; g.ldb = (int)M; g.ldc = (int)M;
              cand.push_back(g);
              fl += 2.0 * (M - oe) * (double)nc * w;
            } else {
              if (ns - oe > 0) {
                GemmTask g{};
                g.A = Lsrc(oe, ob);
                g.B = trow(T, ob);
                g.C = trow(T, oe);
                g.m = (int)(ns - oe); g.n = (int)nc; g.k = (int)w;
                g.lda = (int)ldL; g.ldb = (int)ns; g.ldc = (int)ns;
                cand.push_back(g);
                fl += 2.0 * (ns - oe) * (double)nc * w;
              }
              if (nu > 0) {
                const SNode& q = h->hsn[T.node];
                GemmTask g{};
                g.A = Lsrc(ns, ob);
                g.B = trow(T, ob);
                g.C = scratch + q.Foff + (T.c0 - ns) * nu;
                g.m = (int)nu; g.n = (int)nc; g.k = (int)w;
                g.lda = (int)ldL; g.ldb = (int)ns; g.ldc = (int)nu;
                cand.push_back(g);
                fl += 2.0 * nu * (double)nc * w;
              }
            }
          }
          add_gemm_launch(cand, fl, (int)(ob / 64), K_GEMMO);
        }
        if (ahead && pass == 1) {
          pending.swap(h->fac);
          h->fac.swap(saved);
        }
        }
      }
      for (auto& q : pending) h->fac.push_back(q);
      pending.clear();
    }
  }
  // solves: per level, small fronts by one workgroup each; large fronts (ns > kSolveBigNs)
  // gather + one launch per 64-column block with 256-row chunks per workgroup
  h->fwd.clear();
  h->bwd.clear();
  std::vector<std::vector<Launch>> bwd_levels;
  auto node_of = [&](int64_t s, int64_t b) { return blknode[blkmap.at(s * 1048576 + b)]; };
  auto tri_steps = [&](bool upper, int32_t node, int64_t ob, int64_t oe, std::vector<Launch>& out) {
    const SNode& r = h->hsn[node];
    const int64_t M = (int64_t)r.ns + r.nu, nbs = (r.ns + 63) / 64;
    std::vector<int64_t> jbs;
    for (int64_t jb = ob; jb < oe; jb += 64) jbs.push_back(jb);
    if (upper) std::reverse(jbs.begin(), jbs.end());
    for (int64_t jb : jbs) {
      Launch F;
      F.kind = upper ? K_TRIB : K_TRIF;
      F.step = (int)(upper ? nbs - 1 - jb / 64 : jb / 64);
      F.off = (int64_t)ft.size();
      const int64_t bw = std::min<int64_t>(64, r.ns - jb);
      const int64_t wg = upper ? std::max<int64_t>(1, (jb + 255) / 256) : std::max<int64_t>(1, (M - jb - bw + 255) / 256);
      ft.push_back(FrontTile{node, 0, 0});
      F.cnt = 1;
      F.nwg = wg;
      out.push_back(F);
    }
  };
  // one vector segment of vbuf (doubles [off, off+cnt)) from rank a to rank b, in place
  auto vhop = [&](std::vector<Launch>& seq, std::vector<size_t>& seg, std::vector<int>& cm, int32_t a, int32_t b,
                  int64_t off, int64_t cnt) {
    if (a == b || cnt <= 0 || (h->rank != a && h->rank != b)) return;
    CommOp op;
    const int pi = op.at(h->rank == a ? b : a);
    if (h->rank == a) { op.sbase[pi] = 2; op.soff[pi] = 8 * off; op.sbytes[pi] = 8 * cnt; }
    else { op.rbase[pi] = 2; op.roff[pi] = 8 * off; op.rbytes[pi] = 8 * cnt; }
    add_comm(seq, seg, cm, std::move(op));
  };
  auto holder = [&](int64_t c) { return P.dist(c) ? P.blk_owner(c, P.npblk(c) - 1) : P.owner[c]; };
  constexpr bool no_tiny = false, no_micro = false;
  // large fronts: one sync-free sweep launch per level and direction (default) or one launch per
  // 64-column block (SMLU_SOLVE_STEPS=1, the previous schedule)
  const bool sweep_solve = !tn.solve_steps;
  int64_t ssync_n = 0, ntick = 0;   // flags and ticket counters of the sweep launches
  constexpr int64_t big_work = kSolveBigWork;
  for (int l = 0; l < P.nlevels; ++l) {
    std::vector<int64_t> tiny, small, bigs;
    for (int64_t k = LP[l]; k < LP[l + 1]; ++k) {
      int64_t s = LS[k];
      const SNode& r = h->hsn[s];
      const bool big = r.ns > kSolveBigNs || (int64_t)r.ns * ((int64_t)r.ns + r.nu) > big_work;
      const bool tiny_front = (int64_t)r.ns + r.nu <= kSolveTinyM && r.ns <= 64 && !no_tiny;
      (big ? bigs : tiny_front ? tiny : small).push_back(s);
    }
    std::vector<Launch> bl;
    const size_t fwd0 = h->fwd.size();
    // one GPU: a level's small and tiny fronts are independent of its large fronts (disjoint x rows
    // and front vectors, children in lower levels): they run on the side stream next to the large
    // fronts' gather / sweep chain (solve.cpp)
    const bool overlap = h->nranks == 1 && !bigs.empty() && !(tiny.empty() && small.empty());
    auto mark_level = [&](std::vector<Launch>& seq, size_t from) {
      if (!overlap) return;
      for (size_t i = from; i < seq.size(); ++i) {
        Launch& X = seq[i];
        X.grp = l + 1;
        X.side = X.kind == K_FWDT || X.kind == K_FWD || X.kind == K_BWDT || X.kind == K_BWD;
      }
    };
    // tiny fronts: one wave per front; micro fronts (M <= 8) eight per wave for a single rhs
    for (int micro = 1; micro >= 0; --micro) {
      Launch L;
      L.kind = K_FWDT;
      L.aux = micro;
      L.off = (int64_t)ilist.size();
      for (auto s : tiny)
        if ((P.M(s) <= kSolveMicroM && !no_micro) == (micro == 1)) ilist.push_back((int32_t)s);
      L.cnt = (int64_t)ilist.size() - L.off;
      if (L.cnt == 0) continue;
      h->fwd.push_back(L);
      L.kind = K_BWDT;
      bl.push_back(L);
    }
    if (!small.empty()) {
      Launch L;
      L.kind = K_FWD;
      L.off = (int64_t)ilist.size();
      for (auto s : small) ilist.push_back((int32_t)s);
      L.cnt = (int64_t)small.size();
      h->fwd.push_back(L);
      L.kind = K_BWD;
      bl.push_back(L);
    }
    if (!bigs.empty()) {
      // gather: one thread per front row pulls its own value and the children's contributions (in
      // child order) -- k_fwd_pull; pull lists per front row: gptr (CSR, relative to the front's
      // block) -> gent (vbuf index of each contribution)
      Launch L;
      L.kind = K_FWDP;
      L.off = (int64_t)ft.size();
      int64_t wgp = 0;
      for (auto s : bigs) {
        const SNode& r = h->hsn[s];
        const int64_t M = (int64_t)r.ns + r.nu;
        ft.push_back(FrontTile{(int32_t)s, (int32_t)gptr.size(), wgp});
        wgp += (M + 255) / 256;
        std::vector<int32_t> cnt(M + 1, 0);
        for (int c = r.chbeg; c < r.chend; ++c) {
          const SNode& ch = h->hsn[P.ch_list[c]];
          const int32_t* rm = P.relmap.data() + ch.rowptr;
          for (int32_t k = 0; k < ch.nu; ++k) ++cnt[rm[k] + 1];
        }
        for (int64_t t = 0; t < M; ++t) cnt[t + 1] += cnt[t];
        const int64_t base = (int64_t)gent.size();
        for (int64_t t = 0; t <= M; ++t) gptr.push_back((int32_t)(base + cnt[t]));
        gent.resize(base + cnt[M]);
        for (int c = r.chbeg; c < r.chend; ++c) {
          const SNode& ch = h->hsn[P.ch_list[c]];
          const int32_t* rm = P.relmap.data() + ch.rowptr;
          for (int32_t k = 0; k < ch.nu; ++k) gent[base + cnt[rm[k]]++] = (int32_t)(ch.voff + ch.ns + k);
        }
        if ((int64_t)gptr.size() >= INT32_MAX || (int64_t)gent.size() >= INT32_MAX || r.voff + M >= INT32_MAX)
          return fail(h, SMLU_ERR_ALLOC, "solve gather lists exceed 32-bit indices");
      }
      L.cnt = (int64_t)bigs.size();
      L.nwg = wgp;
      h->fwd.push_back(L);
      int64_t nb = 0;
      for (auto s : bigs) nb = std::max<int64_t>(nb, (h->hsn[s].ns + 63) / 64);
      // backward: U12 product first
      Launch U;
      U.kind = K_BWDU;
      U.off = (int64_t)ft.size();
      int64_t wg = 0;
      for (auto s : bigs) {
        ft.push_back(FrontTile{(int32_t)s, 0, wg});
        wg += (h->hsn[s].ns + 63) / 64;   // k_bwd_u12: 64 rows per workgroup
      }
      U.cnt = (int64_t)bigs.size();
      U.nwg = wg;
      if (sweep_solve) {   // one sync-free sweep launch per direction (k_tri_sweep)
        Launch F, B;
        F.kind = K_SWEEPF;
        B.kind = K_SWEEPB;
        F.off = (int64_t)ft.size();
        F.aux = ssync_n;
        F.aux2 = ntick++;
        int64_t wf = 0;
        int32_t fb = 0;
        for (auto s : bigs) {
          const SNode& r = h->hsn[s];
          ft.push_back(FrontTile{(int32_t)s, fb, wf});
          wf += ((int64_t)r.ns + r.nu + 64 * kSweepWK - 1) / (64 * kSweepWK);
          fb += (r.ns + 63) / 64;
        }
        F.cnt = (int64_t)bigs.size();
        F.nwg = wf;
        ssync_n += fb;
        h->fwd.push_back(F);
        B.off = (int64_t)ft.size();
        B.aux = ssync_n;
        B.aux2 = ntick++;
        int64_t wb = 0;
        fb = 0;
        for (auto s : bigs) {
          const SNode& r = h->hsn[s];
          const int64_t nbs = (r.ns + 63) / 64;
          ft.push_back(FrontTile{(int32_t)s, fb, wb});
          wb += (nbs + kSweepWK - 1) / kSweepWK;
          fb += (int32_t)nbs;
        }
        B.cnt = (int64_t)bigs.size();
        B.nwg = wb;
        ssync_n += fb;
        bl.push_back(U);
        bl.push_back(B);
        mark_level(h->fwd, fwd0);
        mark_level(bl, 0);
        bwd_levels.push_back(bl);
        goto shared_fronts;
      }
      std::vector<Launch> bsteps;
      for (int64_t t = 0; t < nb; ++t) {
        Launch F, B;
        F.kind = K_TRIF;
        B.kind = K_TRIB;
        F.step = B.step = (int)t;
        F.off = (int64_t)ft.size();
        int64_t wf = 0, cnt = 0;
        for (auto s : bigs) {
          const SNode& r = h->hsn[s];
          int64_t nbs = (r.ns + 63) / 64;
          if (t >= nbs) continue;
          int64_t jb = t * 64, bw = std::min<int64_t>(64, r.ns - jb), M = (int64_t)r.ns + r.nu;
          ft.push_back(FrontTile{(int32_t)s, 0, wf});
          wf += std::max<int64_t>(1, (M - jb - bw + 255) / 256);
          ++cnt;
        }
        F.cnt = cnt;
        F.nwg = wf;
        h->fwd.push_back(F);
        B.off = (int64_t)ft.size();
        int64_t wb = 0;
        cnt = 0;
        for (auto s : bigs) {
          const SNode& r = h->hsn[s];
          int64_t nbs = (r.ns + 63) / 64;
          if (t >= nbs) continue;
          int64_t jb = (nbs - 1 - t) * 64;
          ft.push_back(FrontTile{(int32_t)s, 0, wb});
          wb += std::max<int64_t>(1, (jb + 255) / 256);
          ++cnt;
        }
        B.cnt = cnt;
        B.nwg = wb;
        bsteps.push_back(B);
      }
      bl.push_back(U);
      for (auto& b : bsteps) bl.push_back(b);
    }
    mark_level(h->fwd, fwd0);
    mark_level(bl, 0);
    bwd_levels.push_back(bl);
  shared_fronts:
    // forward solve of the shared front: the children's update vectors go to the first block's
    // owner, which gathers the front vector; the vector then follows the pivot blocks' owners
    // (shared fronts of this level, in front order on every rank)
    for (const int32_t t : dfront[l]) {
      const int64_t np = P.npblk(t), M = P.M(t);
      const int64_t tv = h->hsn[t].voff;
      const int32_t o0 = P.blk_owner(t, 0);
      {
        CommOp op;
        std::vector<std::vector<int64_t>> kids(h->nranks);
        for (int64_t e = P.ch_ptr[t]; e < P.ch_ptr[t + 1]; ++e) kids[holder(P.ch_list[e])].push_back(P.ch_list[e]);
        for (int32_t q = 0; q < h->nranks; ++q) {
          if (q == o0 || kids[q].empty()) continue;
          if (h->rank != q && h->rank != o0) continue;
          const int pi = op.at(h->rank == q ? o0 : q);
          int64_t acc = 0;
          for (int64_t c : kids[q]) {
            const int64_t off = 8 * (h->hsn[c].voff + P.ns(c)), nb8 = 8 * P.nu(c);
            if (h->rank == q) op.pack.push_back(HSeg{2, off, 4, acc, nb8});
            else op.unpack.push_back(HSeg{5, acc, 2, off, nb8});
            acc += nb8;
          }
          if (h->rank == q) op.sbytes[pi] = acc;
          else op.rbytes[pi] = acc;
        }
        // receive offsets: per peer contiguous in the receive staging
        int64_t racc = 0;
        for (size_t i = 0; i < op.peer.size(); ++i) {
          op.roff[i] = racc;
          racc += op.rbytes[i];
        }
        if (h->rank == o0) {   // unpack offsets were per peer from 0: shift by the peer's roff
          size_t k = 0;
          for (int32_t q = 0; q < h->nranks; ++q) {
            if (q == o0 || kids[q].empty()) continue;
            int64_t shift = 0;
            for (size_t i = 0; i < op.peer.size(); ++i)
              if (op.peer[i] == q) shift = op.roff[i];
            for (size_t j = 0; j < kids[q].size(); ++j) op.unpack[k++].so += shift;
          }
        }
        if (!op.peer.empty()) add_comm(h->fwd, h->fwd_seg, h->fwd_comm, std::move(op));
      }
      if (h->rank == o0) {
        Launch L;
        L.kind = K_FWDG;
        L.off = (int64_t)ilist.size();
        ilist.push_back(t);
        L.cnt = 1;
        h->fwd.push_back(L);
      }
      for (int64_t b = 0; b < np; ++b) {
        const int32_t o = P.blk_owner(t, b);
        const int64_t ob = P.blk_c0(t, b), oe = P.blk_c1(t, b);
        if (h->rank == o) tri_steps(false, node_of(t, b), ob, oe, h->fwd);
        if (b + 1 < np) vhop(h->fwd, h->fwd_seg, h->fwd_comm, o, P.blk_owner(t, b + 1), tv + oe, M - oe);
      }
    }
  }
  // backward, from the root level down; after each level holding a shared front (and at the
  // end) every rank shares the solution rows it computed since the previous exchange
  std::vector<std::vector<std::pair<int64_t, int64_t>>> pending_rows(h->nranks);   // per rank, since the last exchange
  std::vector<std::pair<int64_t, int64_t>> myrows;   // x rows (first, count) since the last exchange
  auto xbwd = [&]() {
    CommOp op;
    int64_t mine = 0;
    for (auto& rg : myrows) {
      op.pack.push_back(HSeg{3, 8 * rg.first, 4, 8 * mine, 8 * rg.second});
      mine += rg.second;
    }
    // every peer's rows, in its own order (the same enumeration on every rank)
    std::vector<std::vector<std::pair<int64_t, int64_t>>> theirs(h->nranks);
    theirs.swap(pending_rows);
    int64_t racc = 0;
    for (int32_t q = 0; q < h->nranks; ++q) {
      if (q == h->rank) continue;
      const int pi = op.at(q);
      op.soff[pi] = 0;
      op.sbytes[pi] = 8 * mine;
      op.roff[pi] = racc;
      int64_t cnt = 0;
      for (auto& rg : theirs[q]) {
        op.unpack.push_back(HSeg{5, racc + 8 * cnt, 3, 8 * rg.first, 8 * rg.second});
        cnt += rg.second;
      }
      op.rbytes[pi] = 8 * cnt;
      racc += 8 * cnt;
    }
    myrows.clear();
    add_comm(h->bwd, h->bwd_seg, h->bwd_comm, std::move(op));
  };
  (void)xbwd;
  for (int l = P.nlevels - 1; l >= 0; --l) {
    for (auto& L : bwd_levels[l]) h->bwd.push_back(L);
    if (h->nranks == 1) continue;
    // rows every rank computes at this level (global enumeration)
    for (int64_t k = P.lev_ptr[l]; k < P.lev_ptr[l + 1]; ++k) {
      const int64_t s = P.lev_sup[k];
      if (!P.dist(s)) {
        pending_rows[P.owner[s]].push_back({P.s_first[s], P.ns(s)});
        continue;
      }
      for (int64_t b = 0; b < P.npblk(s); ++b)
        pending_rows[P.blk_owner(s, b)].push_back({P.s_first[s] + P.blk_c0(s, b), P.blk_c1(s, b) - P.blk_c0(s, b)});
    }
    // (shared fronts of this level, in front order on every rank)
    for (const int32_t t : dfront[l]) {
      const int64_t np = P.npblk(t), nbk = np + P.nublk(t), ns = P.ns(t);
      const int64_t tv = h->hsn[t].voff;
      // the forward solve left y of each pivot block in x on the block's owner: the rank that
      // starts the backward chain collects all of them first
      const int32_t cs = nbk > np ? P.blk_owner(t, np) : P.blk_owner(t, np - 1);
      {
        CommOp op;
        const int64_t f0 = P.s_first[t];
        for (int32_t q = 0; q < h->nranks; ++q) {
          if (q == cs || (h->rank != q && h->rank != cs)) continue;
          int64_t acc = 0;
          std::vector<HSeg> segs;
          for (int64_t b = 0; b < np; ++b) {
            if (P.blk_owner(t, b) != q) continue;
            const int64_t o8 = 8 * (f0 + P.blk_c0(t, b)), nb8 = 8 * (P.blk_c1(t, b) - P.blk_c0(t, b));
            segs.push_back(h->rank == q ? HSeg{3, o8, 4, acc, nb8} : HSeg{5, acc, 3, o8, nb8});
            acc += nb8;
          }
          if (acc == 0) continue;
          const int pi = op.at(h->rank == q ? cs : q);
          if (h->rank == q) {
            op.sbytes[pi] = acc;
            for (auto& g : segs) op.pack.push_back(g);
          } else {
            op.rbytes[pi] = acc;
            for (auto& g : segs) op.unpack.push_back(g);
          }
        }
        if (h->rank == cs) {   // receive offsets per peer, shift the unpack copies
          int64_t racc = 0;
          size_t k = 0;
          for (size_t i = 0; i < op.peer.size(); ++i) {
            op.roff[i] = racc;
            int64_t left = op.rbytes[i];
            while (left > 0 && k < op.unpack.size()) {
              op.unpack[k].so += racc;
              left -= op.unpack[k].bytes;
              ++k;
            }
            racc += op.rbytes[i];
          }
        }
        if (!op.peer.empty()) add_comm(h->bwd, h->bwd_seg, h->bwd_comm, std::move(op));
      }
      int32_t prev = -1;
      bool first = true;
      for (int64_t ub = np; ub < nbk; ++ub) {   // U12 contributions, block by block
        const int32_t o = P.blk_owner(t, ub);
        if (prev >= 0) vhop(h->bwd, h->bwd_seg, h->bwd_comm, prev, o, tv, ns);
        if (h->rank == o) {
          Launch L;
          L.kind = K_BWDU12C;
          L.node = node_of(t, ub);
          L.aux = P.blk_c0(t, ub);
          L.aux2 = P.blk_c1(t, ub);
          L.cnt = first ? 1 : 0;
          h->bwd.push_back(L);
        }
        prev = o;
        first = false;
      }
      if (first) {   // no update columns: the chain starts from the solution rows of the front
        prev = P.blk_owner(t, np - 1);
        if (h->rank == prev) {
          Launch L;
          L.kind = K_VCOPY;
          L.node = t;
          h->bwd.push_back(L);
        }
      }
      for (int64_t b = np - 1; b >= 0; --b) {
        const int32_t o = P.blk_owner(t, b);
        const int64_t ob = P.blk_c0(t, b), oe = P.blk_c1(t, b);
        vhop(h->bwd, h->bwd_seg, h->bwd_comm, prev, o, tv, oe);
        if (h->rank == o) tri_steps(true, node_of(t, b), ob, oe, h->bwd);
        prev = o;
      }
    }
    for (auto& rg : pending_rows[h->rank]) myrows.push_back(rg);
    pending_rows[h->rank].clear();
    if (dlevel[l] || l == 0) xbwd();
  }

  h->nlaunch = (int64_t)h->fac.size();
  // upload
  if (!h->host_only) {
    HIPCHK(h->sn.upload(h->hsn.data(), h->hsn.size(), st));
    HIPCHK(h->ilist.upload(ilist.data(), ilist.size(), st));
    HIPCHK(h->xtasks.upload(xt.data(), xt.size(), st));
    HIPCHK(h->aents.upload(ae.data(), ae.size(), st));
  }
  // batched right-hand sides (one GPU): the sweep's single chain wave per block would run the NR
  // chains one after another, so batches keep the per-64-column-block launches (k_tri_block: the
  // diagonal block solved by four chain waves for four right-hand sides at a time).  The same
  // per-block sequences (with the comm segments of fwd / bwd) re-run a solve whose sweep timed out.
  h->fwdm.clear();
  h->bwdm.clear();
  {
    auto expand = [&](const Launch& S, bool upper, std::vector<Launch>& out) {
      std::vector<int32_t> fr;
      for (int64_t i = S.off; i < S.off + S.cnt; ++i) fr.push_back(ft[i].s);
      int64_t nb = 0;
      for (auto s : fr) nb = std::max<int64_t>(nb, (h->hsn[s].ns + 63) / 64);
      for (int64_t t = 0; t < nb; ++t) {
        Launch F;
        F.kind = upper ? K_TRIB : K_TRIF;
        F.grp = S.grp;
        F.step = (int)t;
        F.off = (int64_t)ft.size();
        int64_t w = 0, cnt = 0;
        for (auto s : fr) {
          const SNode& r = h->hsn[s];
          const int64_t nbs = (r.ns + 63) / 64, M = (int64_t)r.ns + r.nu;
          if (t >= nbs) continue;
          const int64_t jb = upper ? (nbs - 1 - t) * 64 : t * 64, bw = std::min<int64_t>(64, r.ns - jb);
          ft.push_back(FrontTile{s, 0, w});
          w += upper ? std::max<int64_t>(1, (jb + 255) / 256) : std::max<int64_t>(1, (M - jb - bw + 255) / 256);
          ++cnt;
        }
        F.cnt = cnt;
        F.nwg = w;
        out.push_back(F);
      }
    };
    auto expand_all = [&](const std::vector<Launch>& in, const std::vector<size_t>& seg, bool upper,
                          std::vector<Launch>& out, std::vector<size_t>& oseg) {
      std::vector<size_t> at(in.size() + 1);
      for (size_t i = 0; i < in.size(); ++i) {
        at[i] = out.size();
        if (in[i].kind == (upper ? K_SWEEPB : K_SWEEPF)) expand(in[i], upper, out);
        else out.push_back(in[i]);
      }
      at[in.size()] = out.size();
      oseg.clear();
      for (size_t k : seg) oseg.push_back(at[std::min(k, in.size())]);
    };
    expand_all(h->fwd, h->fwd_seg, false, h->fwdm, h->fwdm_seg);
    expand_all(h->bwd, h->bwd_seg, true, h->bwdm, h->bwdm_seg);
  }
  if (h->nranks > 1) max_list = std::max<int64_t>(max_list, dist_slots);
  h->ssync_n = ssync_n;
  if (h->host_only) {   // smlu_plan_rank_schedule: the schedule without a device
    int64_t ss, rs, hs, hr;
    stage_sizes(h, ss, rs, hs, hr);
    int64_t nseg = 0;
    for (const CommOp& op : h->comm) nseg += (int64_t)(op.pack.size() + op.unpack.size());
    h->host_bytes[3] += 8.0 * ((ss + 7) / 8 + 1) + 8.0 * ((rs + 7) / 8 + 1);   // device staging
    h->host_bytes[0] += h->host_bytes[3];
    h->host_bytes[0] += sizeof(SNode) * (double)h->hsn.size() + 4.0 * ilist.size() + sizeof(XContrib) * (double)xt.size() +
                        sizeof(int2) * (double)ae.size() + sizeof(FrontTile) * (double)ft.size() +
                        4.0 * (gptr.size() + gent.size()) + 4.0 * ssync_n + 8.0 * ntick +
                        8.0 * 64 * kMultiRhs * ssync_n + 4.0 +
                        ((!tinv_patch.empty() || h->nranks > 1) ? 8.0 * 8192 * max_list : 0.0) +
                        sizeof(GemmTask) * (double)gt.size() + sizeof(SwapTask) * (double)st_tasks.size() +
                        sizeof(URowTask) * (double)ur_tasks.size() + sizeof(XCol) * (double)xc.size() +
                        4.0 * kSwapStride * max_list + 8.0 * std::max<int64_t>(voff, 1) + sizeof(SegDesc) * (double)nseg;
    h->host_bytes[4] = (double)hs + (double)hr;   // pinned host staging of a host-memory transport
    return SMLU_OK;
  }
  HIPCHK(h->ftiles.upload(ft.data(), ft.size(), st));
  if (!gptr.empty()) {
    HIPCHK(h->gptr.upload(gptr.data(), gptr.size(), st));
    HIPCHK(h->gent.upload(gent.data(), gent.size(), st));
  }
  if (ssync_n > 0) {   // zeroed once per schedule: the sweeps never reset them (epochs, kernels_solve.hip)
    HIPCHK(h->ssync.alloc((size_t)ssync_n));
    HIPCHK(h->stick.alloc((size_t)ntick));
    HIPCHK(h->sxh.alloc((size_t)ssync_n * 64 * kMultiRhs));
    {   // hand-off slots start as the sweep's sentinel (kernels_solve.hip: k_tri_sweep)
      const long long sent = 0x7ff4dead5eed0001ll;
      double sv;
      std::memcpy(&sv, &sent, sizeof sv);
      HIPCHK(launch_fill(st, ssync_n * 64 * kMultiRhs, h->sxh.p, sv));
    }
    HIPCHK(hipMemsetAsync(h->ssync.p, 0, sizeof(int32_t) * ssync_n, st));
    HIPCHK(hipMemsetAsync(h->stick.p, 0, sizeof(unsigned long long) * ntick, st));
    HIPCHK(hipStreamSynchronize(st));
  }
  if (!h->sstatus.p) {
    HIPCHK(h->sstatus.alloc(1));
    HIPCHK(hipMemsetAsync(h->sstatus.p, 0, sizeof(int32_t), st));
  }
  h->sweep_spin = tn.sweep_spin;
  if (!tinv_patch.empty() || h->nranks > 1) {   // operands in the tile-inverse slots: patch in the buffer address
    HIPCHK(h->tinv.alloc((size_t)max_list * 8192));
    for (auto& pt : tinv_patch) {
      const double* a = h->tinv.p + pt.second / 2;
      if (pt.second & 1) gt[pt.first].B = a;
      else gt[pt.first].A = a;
    }
  }
  HIPCHK(h->gtasks.upload(gt.data(), gt.size(), st));
  HIPCHK(h->stasks.upload(st_tasks.data(), st_tasks.size(), st));
  HIPCHK(h->urtasks.upload(ur_tasks.data(), ur_tasks.size(), st));
  HIPCHK(h->xcols.upload(xc.data(), xc.size(), st));
  HIPCHK(h->swaps.alloc((size_t)max_list * kSwapStride));
  HIPCHK(h->vbuf.alloc((size_t)std::max<int64_t>(voff, 1)));
  // communication steps: staging sizes, then every pack / unpack copy as a device descriptor
  if (!h->comm.empty()) {
    int64_t ss, rs, hs, hr;
    stage_sizes(h, ss, rs, hs, hr);
    h->stage_bytes_s = ss;
    h->stage_bytes_r = rs;
    HIPCHK(h->stage_s.alloc((size_t)(ss + 7) / 8 + 1));
    HIPCHK(h->stage_r.alloc((size_t)(rs + 7) / 8 + 1));
    if (!h->tr.device_memory) {
      HIPCHK(hipHostMalloc((void**)&h->hstage_s, (size_t)std::max<int64_t>(hs, 8), 0));
      HIPCHK(hipHostMalloc((void**)&h->hstage_r, (size_t)std::max<int64_t>(hr, 8), 0));
    }
    char* base[10] = {(char*)h->store.p, (char*)h->scratch.p, (char*)h->vbuf.p, (char*)h->wrk.p,
                      (char*)h->stage_s.p, (char*)h->stage_r.p, (char*)h->bcbuf.p, (char*)h->tinv.p,
                      (char*)h->swaps.p, (char*)h->rowperm.p};
    std::vector<SegDesc> d;
    for (CommOp& op : h->comm) {
      auto emit = [&](const std::vector<HSeg>& v, int64_t& at) {
        at = (int64_t)d.size();
        for (const HSeg& g : v)
          d.push_back(SegDesc{(uint64_t)(base[g.sb] + g.so), (uint64_t)(base[g.db] + g.dof), g.bytes / 4});
      };
      emit(op.pack, op.pack0);
      emit(op.unpack, op.unpack0);
    }
    HIPCHK(h->segdesc.upload(d.data(), d.size(), st));
  }
  HIPCHK(hipStreamSynchronize(st));
  return SMLU_OK;
}

// This rank's layout: the plan's own on one GPU; ordinary fronts + owned column blocks of the
// shared fronts on a partitioned handle.
static void rank_layout_of(smlu_handle* h) {
  const Plan& P = h->plan;
  if (h->nranks > 1) {
    rank_layout(P, h->rank, h->lay);
  } else {
    RankLayout& Y = h->lay;
    Y = RankLayout();
    Y.Loff = P.Loff;
    Y.Uoff = P.Uoff;
    Y.Foff = P.Foff;
    Y.recv_off.assign(P.nsup, -1);
    Y.recv_size.assign(P.nsup, 0);
    Y.store_size = P.factor_size;
    Y.scratch_size = P.scratch_size;
  }
}

// Element counts of the large per-handle buffers (doubles).
struct Sizes {
  int64_t store, scratch, bcbuf;
};
static Sizes sizes_of(const smlu_handle* h) {
  const Plan& P = h->plan;
  Sizes z{};
  // k_urows reads up to 64 columns and 16 rows past a block (values discarded): pad the store
  int64_t maxM = 1;
  for (int64_t s = 0; s < P.nsup; ++s) maxM = std::max<int64_t>(maxM, P.M(s));
  z.store = std::max<int64_t>(h->lay.store_size, 1) + 64 * maxM + 4096;
  z.scratch = std::max<int64_t>(h->lay.scratch_size, 1);
  z.bcbuf = 0;
  if (h->nranks > 1) {   // received pivot block + tile inverses + swap lists + rowperm
    z.bcbuf = 1;
    for (int64_t s = 0; s < P.nsup; ++s)
      if (P.dist(s) && std::binary_search(P.group[s].begin(), P.group[s].end(), h->rank))
        z.bcbuf = std::max<int64_t>(z.bcbuf, P.M(s) * P.dob + (P.dob / 64) * 8192 + (P.dob / 64) * kSwapStride / 2 + P.dob / 2 + 64);
  }
  return z;
}

// Host-only build of a rank's schedule (smlu_plan_rank_schedule): the launch sequences and the
// communication steps exactly as setup_device builds them, no device and no stream.  host_bytes:
// [0] device bytes the handle would allocate, [1] factor store, [2] front scratch, [3] staging +
// received-block buffer, [4] pinned host staging (host-memory transports).
int build_schedule_host(smlu_handle* h) {
  const Plan& P = h->plan;
  h->host_only = true;
  rank_layout_of(h);
  const Sizes z = sizes_of(h);
  const double n = (double)P.n, nnzA = (double)P.nnzA;
  for (double& b : h->host_bytes) b = 0;
  h->host_bytes[1] = 8.0 * z.store;
  h->host_bytes[2] = 8.0 * z.scratch;
  h->host_bytes[3] = 8.0 * z.bcbuf + (h->nranks > 1 ? 64.0 : 0.0);
  h->nnodes = P.nsup + (int64_t)h->lay.blocks.size();
  // A, Rs, wrk, wrk2, growth, Arowptr, Arow_ent, Arow, p0, q, rows, relmap, chlist, posfirst,
  // rowperm, rowperm0, info, status record
  h->host_bytes[0] = h->host_bytes[1] + h->host_bytes[2] + 8.0 * nnzA + 8.0 * n * 3 + 8.0 + 8.0 * (n + 1) +
                     4.0 * nnzA * 2 + 8.0 * n * 3 + 4.0 * (double)(P.s_rows.size() + P.relmap.size() + P.ch_list.size()) +
                     4.0 * n * 2 + 4.0 * (double)h->nnodes + 8.0 * (16 + 5 * 512);
  return build_schedule(h);
}

int setup_device(smlu_handle* h) {
  Plan& P = h->plan;
  HIPCHK(hipSetDevice(h->device));
  // one high-priority stream per handle (the schedule is one stream-ordered sequence)
  int prio_lo = 0, prio_hi = 0;
  HIPCHK(hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi));
  if (!h->stream) HIPCHK(hipStreamCreateWithPriority(&h->stream, hipStreamNonBlocking, prio_hi));
  if (!h->side) HIPCHK(hipStreamCreateWithPriority(&h->side, hipStreamNonBlocking, prio_hi));
  if (!h->fork_ev) HIPCHK(hipEventCreateWithFlags(&h->fork_ev, hipEventDisableTiming));
  if (!h->join_ev) HIPCHK(hipEventCreateWithFlags(&h->join_ev, hipEventDisableTiming));
  hipStream_t st = h->stream;
  rank_layout_of(h);
  const Sizes z = sizes_of(h);
  HIPCHK(h->A.alloc((size_t)std::max<int64_t>(P.nnzA, 1)));
  HIPCHK(h->Rs.alloc((size_t)P.n));
  HIPCHK(h->store.alloc((size_t)z.store));
  HIPCHK(h->scratch.alloc((size_t)z.scratch));
  if (h->nranks > 1) {
    HIPCHK(h->bcbuf.alloc((size_t)z.bcbuf));
    HIPCHK(h->d_red.alloc(8));
  }
  HIPCHK(h->wrk.alloc((size_t)P.n));
  HIPCHK(h->wrk2.alloc((size_t)P.n));
  HIPCHK(h->growth.alloc(2));   // [0] growth maximum, [1] dominance flags (factor.cpp)
  HIPCHK(h->Arowptr.upload(P.Arowptr.data(), P.Arowptr.size(), st));
  HIPCHK(h->Arow_ent.upload(P.Arow_ent.data(), P.Arow_ent.size(), st));
  HIPCHK(h->Arow.upload(P.Arow.data(), P.Arow.size(), st));
  HIPCHK(h->p0.upload(P.p0.data(), P.p0.size(), st));
  HIPCHK(h->q.upload(P.q.data(), P.q.size(), st));
  HIPCHK(h->rows.upload(P.s_rows.data(), P.s_rows.size(), st));
  HIPCHK(h->relmap.upload(P.relmap.data(), P.relmap.size(), st));
  HIPCHK(h->chlist.upload(P.ch_list.data(), P.ch_list.size(), st));
  std::vector<int64_t> pf(P.n);
  for (int64_t s = 0; s < P.nsup; ++s)
    for (int64_t j = P.s_first[s]; j < P.s_first[s + 1]; ++j) pf[j] = P.s_first[s];
  HIPCHK(h->posfirst.upload(pf.data(), pf.size(), st));
  HIPCHK(h->rowperm.alloc((size_t)P.n));
  {
    std::vector<int32_t> id(P.n);
    for (int64_t j = 0; j < P.n; ++j) id[j] = (int32_t)(j - pf[j]);
    HIPCHK(h->rowperm0.upload(id.data(), id.size(), st));
  }
  const int64_t nnodes = P.nsup + (int64_t)h->lay.blocks.size();
  HIPCHK(h->info.alloc((size_t)std::max<int64_t>(nnodes, 1)));
  HIPCHK(init_kernel_attributes());
  if (!h->rb.p) HIPCHK(h->rb.alloc(16 + 5 * 512));   // record + k_status_part's partials
  return build_schedule(h);
}


// Schedule-dependent device buffers and graphs (rebuilt when the pivoting mode changes).
static void release_schedule(smlu_handle* h) {
  h->release_graphs();
  h->sn.free();
  h->ilist.free();
  h->xtasks.free();
  h->aents.free();
  h->ftiles.free();
  h->gptr.free();
  h->gent.free();
  h->ssync.free();
  h->stick.free();
  h->sxh.free();
  h->gtasks.free();
  h->stasks.free();
  h->urtasks.free();
  h->xcols.free();
  h->swaps.free();
  h->vbuf.free();
  h->vbufm.free();
  h->tinv.free();
  h->stage_s.free();
  h->stage_r.free();
  h->segdesc.free();
  if (h->hstage_s) (void)hipHostFree(h->hstage_s);
  if (h->hstage_r) (void)hipHostFree(h->hstage_r);
  h->hstage_s = h->hstage_r = nullptr;
}

int rebuild_schedule(smlu_handle* h) {
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(hipStreamSynchronize(h->stream));
  release_schedule(h);
  return build_schedule(h);
}

bool has_tile_fronts(const smlu_handle* h) {
  for (const SNode& r : h->hsn)
    if (r.mode == 2) return true;
  return false;
}

// One numeric factorization with the re-pivoting fallback (UMFPACK re-pivots in
// every lu!, src/SharedMemSparseLU.jl:247): the diagonal-tile pivoting of large fronts only
// searches the 64x64 diagonal tile.  When it meets a zero pivot (the matrix may still be
// nonsingular: a zero diagonal block) or accepts weak pivots, the same values are factored
// again with full-candidate pivoting (every fully-summed row of the front) in every blocked
// front, and the handle keeps that mode until a refactor's host values are diagonally dominant
// again.  A given (p, q) is never re-pivoted.
