"""Multi-GPU sparse LU: one process per GPU, the assembly tree partitioned across ranks.

Replaces the reference's MPI shared-memory column split (src/SharedMemSparseLU.jl:101-160, the
rank split intended at :107 and :128).  libsmlu.so owns the whole partitioned
factorization and solve (include/smlu.h, "multi-GPU partition"): subtrees of the assembly tree
per rank with no communication, the fronts above them shared by their ranks as a 1D
block-cyclic column partition (block owner factors and broadcasts, every member updates its own
column blocks), the children's F22 columns moved to the owners of the parent's columns.  The
library drives every transfer itself through a transport:

* ``nccl`` process group -> the library's built-in RCCL transport (xGMI point-to-point,
  stream-ordered, no host synchronisation): rank 0 draws the RCCL unique id, torch.distributed
  only broadcasts those 128 bytes once;
* ``gloo`` process group -> a host-memory transport implemented here with torch.distributed
  point-to-point calls (tests; several ranks may then share one GPU); ``transport="device"`` runs
  the library's device-memory (RCCL) calling convention over gloo instead.

    F = DistributedSparseLU(A, device=local_rank)   # analysis + allocation + first factorization
    F.refactor_device(d_values)                     # lu!(F, A), values already in HBM (collective)
    F.solve_device(d_x, d_b)                        # ldiv!(x, F, b); x complete on every rank
"""
from __future__ import annotations

import ctypes
import traceback

import numpy as np

from . import _lib as C
from .api import SingularException, SmluError, _csc


def _check(rc, h=None):
    if rc < 0:
        raise SmluError(f"libsmlu error {rc}: {C.last_error(h)}")
    return rc


class HostTransport:
    """smlu_transport over torch.distributed point-to-point calls on host buffers (gloo)."""

    def __init__(self, dist, group=None):
        import torch
        self.torch, self.dist, self.group = torch, dist, group
        self._cb = (C.EXCHANGE_FN(self._exchange), C.BCAST_FN(self._bcast), C.ALLREDUCE_FN(self._allreduce))
        self.struct = C.SmluTransport(None, 0, *self._cb)

    def _view(self, addr, nbytes):
        return self.torch.frombuffer((ctypes.c_uint8 * int(nbytes)).from_address(addr), dtype=self.torch.uint8)

    def _exchange(self, ctx, npeer, peer, sbuf, sbytes, rbuf, rbytes, stream):
        try:
            works = []
            for i in range(npeer):
                if sbytes[i] > 0:
                    works.append(self.dist.isend(self._view(sbuf[i], sbytes[i]), int(peer[i]), group=self.group))
                if rbytes[i] > 0:
                    works.append(self.dist.irecv(self._view(rbuf[i], rbytes[i]), int(peer[i]), group=self.group))
            for w in works:
                w.wait()
            return 0
        except Exception:
            traceback.print_exc()
            return 1

    def _bcast(self, ctx, buf, nbytes, root, gsize, group, stream):
        try:
            me = self.dist.get_rank(self.group)
            t = self._view(buf, nbytes)
            if me == root:
                works = [self.dist.isend(t, int(group[i]), group=self.group) for i in range(gsize)
                         if int(group[i]) != root]
            else:
                works = [self.dist.irecv(t, int(root), group=self.group)]
            for w in works:
                w.wait()
            return 0
        except Exception:
            traceback.print_exc()
            return 1

    def _allreduce(self, ctx, buf, count):
        try:
            a = np.ctypeslib.as_array(buf, shape=(count,))
            t = self.torch.from_numpy(a.copy())
            self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX, group=self.group)
            a[:] = t.numpy()
            return 0
        except Exception:
            traceback.print_exc()
            return 1


class DeviceStagedTransport(HostTransport):
    """The built-in RCCL transport's calling convention carried over gloo: device_memory = 1, so the
    library hands over DEVICE buffers (its send / receive staging, the broadcast block buffer) on
    its stream, exactly as it does to rccl_exchange / rccl_bcast, and does no host staging of its
    own; each call here synchronises that stream, copies the messages to host memory, moves them
    over gloo and copies the received ones back.  A one-GPU rehearsal of exec_comm's device-memory
    path (the addressing RCCL sees) -- RCCL itself refuses two ranks on one GPU."""

    def __init__(self, dist, group=None):
        super().__init__(dist, group)
        self.struct = C.SmluTransport(None, 1, *self._cb)
        hip = ctypes.CDLL("libamdhip64.so")
        hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        hip.hipMemcpy.restype = ctypes.c_int
        hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
        hip.hipStreamSynchronize.restype = ctypes.c_int
        self.hip = hip

    def _sync(self, stream):
        if self.hip.hipStreamSynchronize(stream) != 0:
            raise RuntimeError("hipStreamSynchronize failed")

    def _d2h(self, dev, n):
        buf = np.empty(int(n), np.uint8)
        if self.hip.hipMemcpy(buf.ctypes.data, dev, int(n), 2) != 0:   # hipMemcpyDeviceToHost
            raise RuntimeError("hipMemcpy D2H failed")
        return buf

    def _h2d(self, dev, buf):
        if self.hip.hipMemcpy(dev, buf.ctypes.data, buf.size, 1) != 0:   # hipMemcpyHostToDevice
            raise RuntimeError("hipMemcpy H2D failed")

    def _exchange(self, ctx, npeer, peer, sbuf, sbytes, rbuf, rbytes, stream):
        try:
            self._sync(stream)
            works, recvs = [], []
            for i in range(npeer):
                if sbytes[i] > 0:
                    works.append(self.dist.isend(self.torch.from_numpy(self._d2h(sbuf[i], sbytes[i])),
                                                 int(peer[i]), group=self.group))
                if rbytes[i] > 0:
                    h = np.empty(int(rbytes[i]), np.uint8)
                    recvs.append((rbuf[i], h))
                    works.append(self.dist.irecv(self.torch.from_numpy(h), int(peer[i]), group=self.group))
            for w in works:
                w.wait()
            for dev, h in recvs:
                self._h2d(dev, h)
            return 0
        except Exception:
            traceback.print_exc()
            return 1

    def _bcast(self, ctx, buf, nbytes, root, gsize, group, stream):
        try:
            self._sync(stream)
            me = self.dist.get_rank(self.group)
            if me == root:
                h = self._d2h(buf, nbytes)
                works = [self.dist.isend(self.torch.from_numpy(h), int(group[i]), group=self.group)
                         for i in range(gsize) if int(group[i]) != root]
                for w in works:
                    w.wait()
            else:
                h = np.empty(int(nbytes), np.uint8)
                self.dist.irecv(self.torch.from_numpy(h), int(root), group=self.group).wait()
                self._h2d(buf, h)
            return 0
        except Exception:
            traceback.print_exc()
            return 1


class DistributedSparseLU:
    """ParallelSparseLU over the ranks of a torch.distributed process group (collective)."""

    def __init__(self, A, *, group=None, device=None, ordering="auto", transport="auto", **opts):
        import torch
        import torch.distributed as dist
        self.torch, self.dist, self.group = torch, dist, group
        self.rank = dist.get_rank(group)
        self.nranks = dist.get_world_size(group)
        backend = dist.get_backend(group)
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None else device)
        A = _csc(A)
        if np.iscomplexobj(A.data):   # the partitioned path is real-only; never drop the imaginary part
            raise TypeError("DistributedSparseLU factors real matrices only (ComplexF64: one GPU)")
        self.n = A.shape[0]
        order = {"auto": C.ORDER_AUTO, "natural": C.ORDER_NATURAL, "nd": C.ORDER_GRAPH_ND,
                 "geometric": C.ORDER_GEOMETRIC_ND, "amd": C.ORDER_AMD}[ordering]
        o = C.default_opts(index_base=0, ordering=order, device=self.device.index, **opts)
        self._colptr = np.ascontiguousarray(A.indptr, dtype=np.int64)
        self._rowval = np.ascontiguousarray(A.indices, dtype=np.int64)
        vals = np.ascontiguousarray(A.data, dtype=np.float64)
        h = ctypes.c_void_p()
        L = C.lib()
        use_rccl = transport == "rccl" or (transport == "auto" and backend == "nccl")
        self.transport = "rccl" if use_rccl else "device" if transport == "device" else "host"
        if use_rccl:
            uid = np.zeros(128, np.uint8)
            if self.rank == 0:
                _check(L.smlu_rccl_unique_id(C.ptr(uid)))
            t = torch.from_numpy(uid)
            if backend == "nccl":
                t = t.to(self.device)
            dist.broadcast(t, 0, group=group)
            uid = np.ascontiguousarray(t.cpu().numpy())
            rc = L.smlu_dist_create_rccl(self.n, C.ptr(self._colptr), C.ptr(self._rowval), C.ptr(vals),
                                         ctypes.byref(o), self.rank, self.nranks, C.ptr(uid), ctypes.byref(h))
        else:   # "host": host-memory transport; "device": the RCCL calling convention over gloo
            self._tr = DeviceStagedTransport(dist, group) if transport == "device" else HostTransport(dist, group)
            rc = L.smlu_dist_create(self.n, C.ptr(self._colptr), C.ptr(self._rowval), C.ptr(vals),
                                    ctypes.byref(o), self.rank, self.nranks, ctypes.byref(self._tr.struct),
                                    ctypes.byref(h))
        if rc < 0:
            raise SmluError(f"smlu_dist_create failed ({rc}): {C.last_error(h if h.value else None)}")
        self._h = h
        self.status = rc
        if rc == C.SMLU_SINGULAR:
            col = L.smlu_last_error_col(h)
            self.close()
            raise SingularException(col)

    @property
    def weak(self):
        return int(self.stat("weak"))

    @property
    def refine_steps(self):
        return int(self.stat("refine_steps"))

    def refactor(self, values):
        """lu!(F, A) with host values (A's CSC order, float64); collective (smlu_refactor)."""
        v = np.ascontiguousarray(values, dtype=np.float64)
        rc = _check(C.lib().smlu_refactor(self._h, C.ptr(v)), self._h)
        self.status = rc
        if rc == C.SMLU_SINGULAR:
            raise SingularException(C.lib().smlu_last_error_col(self._h))
        return rc

    def refactor_device(self, d_values):
        """lu!(F, A) with values already in HBM (A's CSC order); collective."""
        ptr = d_values.data_ptr() if hasattr(d_values, "data_ptr") else int(d_values)
        with C.caller_stream(self._h, d_values):
            rc = _check(C.lib().smlu_refactor_device(self._h, ctypes.c_void_p(ptr)), self._h)
        self.status = rc
        if rc == C.SMLU_SINGULAR:
            raise SingularException(C.lib().smlu_last_error_col(self._h))
        return rc

    def solve_device(self, d_x, d_b):
        """ldiv!(x, F, b) on device vectors; collective; x complete on every rank.  Weak pivots
        anywhere in the partition trigger the same iterative refinement as on one GPU."""
        px = d_x.data_ptr() if hasattr(d_x, "data_ptr") else int(d_x)
        pb = d_b.data_ptr() if hasattr(d_b, "data_ptr") else int(d_b)
        with C.caller_stream(self._h, d_b):
            _check(C.lib().smlu_solve_device(self._h, ctypes.c_void_p(pb), ctypes.c_void_p(px)), self._h)
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
