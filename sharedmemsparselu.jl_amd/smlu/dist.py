"""Multi-GPU sparse LU: one process per GPU, the assembly tree split across ranks.

Replaces the reference's MPI shared-memory column split (src/SharedMemSparseLU.jl:101-160,
ranks own column chunks of one dense-chunk layout).  Here each rank factors the
subtrees that proportional mapping gives it, with no communication; right before the level of
a front whose child lives on another rank, the child's update block (F22) is moved to the
front's owner.  The library (libsmlu.so, `smlu_dist_*`) runs the segments between those
exchange points on its own HIP stream and packs/unpacks the crossing blocks; this module moves
them with torch.distributed: RCCL point-to-point (`nccl` backend, device buffers over xGMI),
or `gloo` through host memory (tests; several ranks may then share one GPU).

    F = DistributedSparseLU(A, device=local_rank)     # analysis + upload, then first factor
    F.refactor_device(d_values)                       # lu!(F, A), values already in HBM
    F.solve_device(d_x, d_b)                          # ldiv!(x, F, b); x complete on every rank
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib as C
from .api import SingularException, SmluError, _csc


def _check(rc, h=None):
    if rc < 0:
        raise SmluError(f"libsmlu error {rc}: {C.last_error(h)}")
    return rc


class DistributedSparseLU:
    def __init__(self, A, *, group=None, device=None, ordering="auto", factor=True, **opts):
        import torch
        import torch.distributed as dist
        self.torch, self.dist, self.group = torch, dist, group
        self.rank = dist.get_rank(group)
        self.nranks = dist.get_world_size(group)
        self.backend = dist.get_backend(group)
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None else device)
        A = _csc(A)
        self.n = A.shape[0]
        order = {"auto": C.ORDER_AUTO, "natural": C.ORDER_NATURAL, "nd": C.ORDER_GRAPH_ND,
                 "geometric": C.ORDER_GEOMETRIC_ND}[ordering]
        o = C.default_opts(index_base=0, ordering=order, device=self.device.index, **opts)
        self._colptr = np.ascontiguousarray(A.indptr, dtype=np.int64)
        self._rowval = np.ascontiguousarray(A.indices, dtype=np.int64)
        vals = np.ascontiguousarray(A.data, dtype=np.float64)
        h = ctypes.c_void_p()
        rc = C.lib().smlu_dist_create(self.n, C.ptr(self._colptr), C.ptr(self._rowval), C.ptr(vals),
                                      ctypes.byref(o), self.rank, self.nranks, ctypes.byref(h))
        if rc < 0:
            raise SmluError(f"smlu_dist_create failed ({rc}): {C.last_error(None)}")
        self._h = h
        self.nseg = int(C.lib().smlu_dist_nsegments(h))
        self.status = None
        self.weak = 0
        self.refine_steps = 0
        if factor:
            _check(C.lib().smlu_dist_set_values(h, C.ptr(vals), 0), h)
            self._factor()

    # ---- exchanges --------------------------------------------------------------------------
    def _sizes(self, kind, seg):
        s = np.zeros(self.nranks, np.int64)
        r = np.zeros(self.nranks, np.int64)
        _check(C.lib().smlu_dist_xsizes(self._h, kind, seg, C.ptr(s), C.ptr(r)), self._h)
        return s, r

    def _exchange(self, kind, seg):
        torch, dist = self.torch, self.dist
        send, recv = self._sizes(kind, seg)
        if kind == 2:   # every rank's new solution rows to every other rank
            mine = int(send.max()) if self.nranks > 1 else 0
            sbuf = torch.empty(max(mine, 1), dtype=torch.float64, device=self.device)
            if mine:
                _check(C.lib().smlu_dist_pack(self._h, kind, seg, ctypes.c_void_p(sbuf.data_ptr())), self._h)
            rbuf = torch.empty(max(int(recv.sum()), 1), dtype=torch.float64, device=self.device)
            off = 0
            for r in range(self.nranks):
                cnt = mine if r == self.rank else int(recv[r])
                if cnt == 0:
                    continue
                if r == self.rank:
                    self._bcast(sbuf[:cnt], r)
                else:
                    self._bcast(rbuf[off:off + cnt], r)
                    off += cnt
            if off:
                _check(C.lib().smlu_dist_unpack(self._h, kind, seg, ctypes.c_void_p(rbuf.data_ptr())), self._h)
            return
        ns, nr = int(send.sum()), int(recv.sum())
        if ns == 0 and nr == 0:
            return
        sbuf = torch.empty(max(ns, 1), dtype=torch.float64, device=self.device)
        rbuf = torch.empty(max(nr, 1), dtype=torch.float64, device=self.device)
        if ns:
            _check(C.lib().smlu_dist_pack(self._h, kind, seg, ctypes.c_void_p(sbuf.data_ptr())), self._h)
        sends, recvs = [], []
        so = ro = 0
        for r in range(self.nranks):
            if send[r]:
                sends.append((r, sbuf[so:so + int(send[r])]))
                so += int(send[r])
            if recv[r]:
                recvs.append((r, rbuf[ro:ro + int(recv[r])]))
                ro += int(recv[r])
        self._p2p(sends, recvs)
        if nr:
            _check(C.lib().smlu_dist_unpack(self._h, kind, seg, ctypes.c_void_p(rbuf.data_ptr())), self._h)

    def _p2p(self, sends, recvs):
        torch, dist = self.torch, self.dist
        if self.backend == "nccl":   # RCCL: device buffers, point-to-point over xGMI
            ops = [dist.P2POp(dist.isend, t, r, self.group) for r, t in sends]
            ops += [dist.P2POp(dist.irecv, t, r, self.group) for r, t in recvs]
            for w in dist.batch_isend_irecv(ops):
                w.wait()
            torch.cuda.synchronize(self.device)
            return
        # gloo: through host memory
        host = [(r, t.cpu()) for r, t in sends]
        hrecv = [(r, torch.empty(t.numel(), dtype=torch.float64), t) for r, t in recvs]
        works = [dist.isend(t, r, group=self.group) for r, t in host]
        works += [dist.irecv(ht, r, group=self.group) for r, ht, _ in hrecv]
        for w in works:
            w.wait()
        for _, ht, t in hrecv:
            t.copy_(ht)
        torch.cuda.synchronize(self.device)

    def _bcast(self, t, src):
        torch, dist = self.torch, self.dist
        if self.backend == "nccl":
            dist.broadcast(t, src, group=self.group)
            torch.cuda.synchronize(self.device)
            return
        ht = t.cpu()
        dist.broadcast(ht, src, group=self.group)
        if src != self.rank:
            t.copy_(ht)
        torch.cuda.synchronize(self.device)

    # ---- lu! / ldiv! ------------------------------------------------------------------------
    def _factor(self):
        L = C.lib()
        rc = 0
        for seg in range(self.nseg):
            if seg > 0:
                self._exchange(0, seg)
            rc = _check(L.smlu_dist_factor_segment(self._h, seg), self._h)
        # every rank learns whether any rank hit a zero pivot (and where) and how many weak
        # pivots the partition accepted: [singular, weak, zero-pivot column] reduced by MAX/SUM
        torch = self.torch
        sing = float(rc == C.SMLU_SINGULAR)
        col = float(L.smlu_last_error_col(self._h)) if sing else -1.0
        st = torch.tensor([sing, col], dtype=torch.float64)
        wk = torch.tensor([self.stat("weak")], dtype=torch.float64)
        if self.backend == "nccl":
            st, wk = st.to(self.device), wk.to(self.device)
        self.dist.all_reduce(st, op=self.dist.ReduceOp.MAX, group=self.group)
        self.dist.all_reduce(wk, op=self.dist.ReduceOp.SUM, group=self.group)
        self.weak = int(wk.item())
        if st[0].item() > 0:
            self.status = C.SMLU_SINGULAR
            raise SingularException(int(st[1].item()))
        self.status = C.SMLU_PIVOT_WEAK if self.weak > 0 else C.SMLU_OK
        return self.status

    def refactor_device(self, d_values):
        ptr = d_values.data_ptr() if hasattr(d_values, "data_ptr") else int(d_values)
        _check(C.lib().smlu_dist_set_values(self._h, ctypes.c_void_p(ptr), 1), self._h)
        return self._factor()

    def solve_device(self, d_x, d_b, refine=None):
        """ldiv!(x, F, b) across the ranks; x complete on every rank.  As on one GPU
        (smlu_solve*), weak pivots anywhere in the partition trigger up to 3 steps of iterative
        refinement (refine=None), stopping when the residual max-norm stops halving; every rank
        holds A and the whole x, so each computes the same residual."""
        steps = (3 if self.weak > 0 else 0) if refine is None else int(refine)
        if steps == 0:
            return self._solve_once(d_x, d_b)
        torch = self.torch
        b = d_b.clone()                  # d_b may alias d_x
        self._solve_once(d_x, b)
        r = torch.empty_like(b)
        d = torch.empty_like(b)
        nrm = ctypes.c_double()
        prev = float("inf")
        self.refine_steps = 0
        for _ in range(steps):
            _check(C.lib().smlu_residual_device(self._h, ctypes.c_void_p(d_x.data_ptr()),
                                                ctypes.c_void_p(b.data_ptr()),
                                                ctypes.c_void_p(r.data_ptr()), ctypes.byref(nrm)),
                   self._h)
            if nrm.value == 0.0 or nrm.value > 0.5 * prev:
                break
            prev = nrm.value
            self._solve_once(d, r)
            d_x += d
            self.refine_steps += 1
        return d_x

    def _solve_once(self, d_x, d_b):
        L = C.lib()
        pb = ctypes.c_void_p(d_b.data_ptr())
        for seg in range(self.nseg):
            if seg > 0:
                self._exchange(1, seg)
            _check(L.smlu_dist_solve_segment(self._h, pb, None, 0, seg), self._h)
        for seg in range(self.nseg):
            if seg > 0:
                self._exchange(2, seg)
            _check(L.smlu_dist_solve_segment(self._h, None, None, 1, seg), self._h)
        _check(L.smlu_dist_solve_segment(self._h, None, ctypes.c_void_p(d_x.data_ptr()), 2, 0), self._h)
        if self.backend == "nccl":
            self.dist.all_reduce(d_x, group=self.group)
        else:
            hx = d_x.cpu()
            self.dist.all_reduce(hx, group=self.group)
            d_x.copy_(hx)
        return d_x

    def stat(self, key):
        return C.lib().smlu_stat(self._h, key.encode())

    def close(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            C.lib().smlu_destroy(h)
        self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
