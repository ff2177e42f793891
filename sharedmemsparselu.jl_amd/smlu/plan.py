"""Host-only access to the symbolic plan (no GPU needed): ordering, supernodes, levels and the
structural pattern of L.  Used by the CPU test-suite and by bench.py for algorithmic byte and
flop counts."""
from __future__ import annotations

import ctypes

import numpy as np
import scipy.sparse as sp

from . import _lib as C


class Plan:
    def __init__(self, A, ordering="auto", grid=None, relax=True, leaf_size=None):
        A = sp.csc_matrix(A, dtype=np.float64)
        A.sort_indices()
        A.sum_duplicates()
        n = A.shape[0]
        order = {"auto": C.ORDER_AUTO, "natural": C.ORDER_NATURAL, "nd": C.ORDER_GRAPH_ND,
                 "geometric": C.ORDER_GEOMETRIC_ND, "amd": C.ORDER_AMD}[ordering]
        kw = dict(index_base=0, ordering=order, relax=1 if relax else 0)
        if grid is not None:
            kw["grid"] = grid
            if ordering == "auto":
                kw["ordering"] = C.ORDER_GEOMETRIC_ND
        if leaf_size is not None:
            kw["leaf_size"] = int(leaf_size)
        o = C.default_opts(**kw)
        self.n = n
        cp = np.ascontiguousarray(A.indptr, dtype=np.int64)
        ri = np.ascontiguousarray(A.indices, dtype=np.int64)
        h = ctypes.c_void_p()
        rc = C.lib().smlu_plan_create(n, C.ptr(cp), C.ptr(ri), ctypes.byref(o), ctypes.byref(h))
        if rc != 0:
            raise RuntimeError(f"smlu_plan_create failed ({rc}): {C.last_error(None)}")
        self._h = h

    def stat(self, key):
        return C.lib().smlu_plan_stat(self._h, key.encode())

    def q(self):
        q = np.empty(self.n, np.int64)
        C.lib().smlu_plan_pattern(self._h, C.ptr(q), None, None)
        return q

    def L_pattern(self):
        n = self.n
        Lp = np.empty(n + 1, np.int64)
        C.lib().smlu_plan_pattern(self._h, None, C.ptr(Lp), None)
        Li = np.empty(Lp[-1], np.int64)
        C.lib().smlu_plan_pattern(self._h, None, C.ptr(Lp), C.ptr(Li))
        return sp.csc_matrix((np.ones(Li.size), Li, Lp), shape=(n, n))

    def supernodes(self):
        ns = int(self.stat("nsuper"))
        first = np.empty(ns + 1, np.int64)
        parent = np.empty(ns, np.int64)
        level = np.empty(ns, np.int64)
        C.lib().smlu_plan_supernodes(self._h, C.ptr(first), C.ptr(parent), C.ptr(level))
        return first, parent, level

    def fronts(self):
        """Assembly tree for the CPU multifrontal oracle: (first, parent, rowptr, rows, p0)."""
        first, parent, _ = self.supernodes()
        ns = first.size - 1
        rowptr = np.empty(ns + 1, np.int64)
        C.lib().smlu_plan_fronts(self._h, C.ptr(rowptr), None, None)
        rows = np.empty(rowptr[-1], np.int64)
        p0 = np.empty(int(self.stat("n")), np.int64)
        C.lib().smlu_plan_fronts(self._h, C.ptr(rowptr), C.ptr(rows), C.ptr(p0))
        return first, parent, rowptr, rows, p0

    def partition(self, nparts):
        """Owner rank per supernode of an `nparts`-rank partitioned handle (-1: a front shared
        by several ranks as a block-cyclic column partition) and the number of shared fronts."""
        ns = int(self.stat("nsuper"))
        owner = np.empty(ns, np.int32)
        nsh = ctypes.c_int64()
        rc = C.lib().smlu_plan_partition(self._h, int(nparts), C.ptr(owner), ctypes.byref(nsh))
        if rc != 0:
            raise RuntimeError(f"smlu_plan_partition failed ({rc}): {C.last_error(None)}")
        return owner, int(nsh.value)

    def rank_memory(self, nparts, rank):
        """Device bytes rank `rank` of `nparts` allocates: (factor store, scratch, staging)."""
        a, b, c = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        rc = C.lib().smlu_plan_rank_memory(self._h, int(nparts), int(rank), ctypes.byref(a), ctypes.byref(b),
                                           ctypes.byref(c))
        if rc != 0:
            raise RuntimeError(f"smlu_plan_rank_memory failed ({rc}): {C.last_error(None)}")
        return a.value, b.value, c.value

    def rank_schedule(self, nparts, rank):
        """Rank `rank`'s schedule of an `nparts`-rank handle built on the host (no device,
        smlu_plan_rank_schedule): its communication steps in execution order as dicts
        {seq: 'fac' | 'fwd' | 'bwd', type: 'exchange' | 'bcast', root, bytes, peers: [(peer, sbytes,
        rbytes)] or group: [ranks]}, and {device_bytes, store_bytes, scratch_bytes, staging_bytes,
        host_staging_bytes, launches, shared_fronts, owned_blocks}."""
        L = C.lib()
        n = ctypes.c_int64()
        by = np.zeros(5)
        cn = np.zeros(3, np.int64)
        ops = np.empty(1 << 20, np.int64)   # one build when the steps fit (256^3 / 8 ranks: ~2e4 words)
        while True:
            rc = L.smlu_plan_rank_schedule(self._h, int(nparts), int(rank), C.ptr(ops), ops.size, ctypes.byref(n),
                                           C.ptr(by), C.ptr(cn))
            if rc == 0:
                break
            if n.value <= ops.size:
                raise RuntimeError(f"smlu_plan_rank_schedule failed ({rc}): {C.last_error(None)}")
            ops = np.empty(n.value, np.int64)
        steps, k, seqs = [], 0, ("fac", "fwd", "bwd")
        while k < n.value:
            q, typ, root, nbytes, cnt = (int(v) for v in ops[k:k + 5])
            k += 5
            if typ == 1:
                steps.append({"seq": seqs[q], "type": "bcast", "root": root, "bytes": nbytes,
                              "group": [int(v) for v in ops[k:k + cnt]]})
                k += cnt
            else:
                trip = ops[k:k + 3 * cnt].reshape(cnt, 3)
                steps.append({"seq": seqs[q], "type": "exchange",
                              "peers": [(int(a), int(b), int(c)) for a, b, c in trip]})
                k += 3 * cnt
        info = {"device_bytes": by[0], "store_bytes": by[1], "scratch_bytes": by[2], "staging_bytes": by[3],
                "host_staging_bytes": by[4], "launches": int(cn[0]), "shared_fronts": int(cn[1]),
                "owned_blocks": int(cn[2])}
        return steps, info

    def project(self, nparts, tflops=52.0, gbs=100.0, lat_us=20.0):
        """Projected partitioned factorization time (s) and the one-GPU time of the same model."""
        t1 = ctypes.c_double()
        t = C.lib().smlu_plan_project(self._h, int(nparts), float(tflops), float(gbs), float(lat_us),
                                      ctypes.byref(t1))
        return t, t1.value

    def front_flops(self):
        """Dense flops per supernode (the partition's work model)."""
        first, parent, level = self.supernodes()
        L = self.L_pattern()
        ns = np.diff(first).astype(np.float64)
        M = np.diff(L.indptr)[first[:-1]].astype(np.float64)
        S2 = lambda x: x * (x + 1) * (2 * x + 1) / 6.0  # noqa: E731
        return 2 * (S2(M - 1) - S2(M - 1 - ns)) + ns * (M - 1) - ns * (ns - 1) / 2

    def __del__(self):
        try:
            if self._h:
                C.lib().smlu_plan_destroy(self._h)
        except Exception:
            pass
