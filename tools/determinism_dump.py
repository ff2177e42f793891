"""Dev: which fronts' factor values (store) or Schur complements (F22, scratch) depend on the values
factored BEFORE the current ones.  History A: v0, v0; history B: v1, v0 (3D Poisson N^3, in-HBM
values).  Per front up to a tree height, compares L panel + U12 and F22 entrywise.

    python tools/determinism_dump.py N [max_height [min_height]]
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sharedmemsparselu.jl_amd"))

import numpy as np  # noqa: E402


def main():
    import torch
    import smlu
    import smlu._lib as C
    from smlu import matrices as mats
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    hmax = int(sys.argv[2]) if len(sys.argv) > 2 else 99
    hmin = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    A = mats.poisson3d(N)
    n = A.shape[0]
    F = smlu.ParallelSparseLU(A, device=0)
    L = C.lib()
    L.smlu_dev_copy.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p,
                                ctypes.c_void_p]
    L.smlu_dev_copy.restype = ctypes.c_int
    L.smlu_dev_front_offsets.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    L.smlu_dev_front_offsets.restype = ctypes.c_int
    fr = F.fronts()
    first, parent, rowptr, fmode = fr["first"], fr["parent"], fr["rowptr"], fr["mode"]
    ns_, nu_ = np.diff(first), np.diff(rowptr)
    nsup = ns_.size
    height = np.zeros(nsup, np.int64)
    for s in range(nsup):
        if parent[s] >= 0:
            height[parent[s]] = max(height[parent[s]], height[s] + 1)
    off = np.zeros(4 * nsup, np.int64)
    assert L.smlu_dev_front_offsets(F._h, off.ctypes.data) == 0
    off = off.reshape(nsup, 4)
    watch = [s for s in range(nsup) if hmin <= height[s] <= hmax]

    def whole(which):
        n = ctypes.c_int64()
        assert L.smlu_dev_copy(F._h, which, 0, -1, None, ctypes.byref(n)) == 0
        out = np.empty(n.value)
        step = 1 << 27
        for o in range(0, n.value, step):
            c = min(step, n.value - o)
            assert L.smlu_dev_copy(F._h, which, o, c, out[o:].ctypes.data, None) == 0
        return out

    def snapshot():
        st, sc = whole(0), whole(1)
        snap = {}
        for s in watch:
            M, ns, nu = int(off[s, 3]), int(ns_[s]), int(nu_[s])
            lu = np.concatenate([st[off[s, 0]:off[s, 0] + M * ns], st[off[s, 1]:off[s, 1] + ns * nu] if nu else np.empty(0)])
            f22 = sc[off[s, 2]:off[s, 2] + nu * nu] if off[s, 2] >= 0 and nu else np.empty(0)
            snap[s] = (lu, f22)
        return snap

    dev = torch.device("cuda", 0)
    dpos = torch.from_numpy(mats.diag_positions(A)).to(dev)
    base = torch.from_numpy(np.ascontiguousarray(A.data)).to(dev)
    vs = []
    for seed in (47, 48):
        v = base.clone()
        v[dpos] += torch.from_numpy(np.random.default_rng(seed).random(n)).to(dev)
        vs.append(v)
    for trial in range(3):
        F.refactor_device(vs[0])
        F.refactor_device(vs[0])
        SA = snapshot()
        F.refactor_device(vs[1])
        F.refactor_device(vs[0])
        SB = snapshot()
        bad = []
        for s in watch:
            dlu = int((SA[s][0] != SB[s][0]).sum())
            df = int((SA[s][1] != SB[s][1]).sum())
            if dlu or df:
                bad.append((int(height[s]), s, dlu, df))
        bad.sort()
        print(f"N={N} trial {trial}: {len(bad)} of {len(watch)} fronts differ (height {hmin}..{hmax})", flush=True)
        for h, s, dlu, df in bad[:10]:
            print(f"   front {s}: height {h} mode {fmode[s]} ns {ns_[s]} nu {nu_[s]}: L/U entries {dlu}, F22 entries {df}; "
                  f"children {[int(c) for c in np.nonzero(parent == s)[0]][:8]}", flush=True)
        if bad:
            h, s, dlu, df = bad[0]
            M, ns = int(off[s, 3]), int(ns_[s])
            a, b = SA[s][1], SB[s][1]
            d = np.nonzero(a != b)[0]
            if d.size:
                nu = int(nu_[s])
                print(f"   first front's F22 diffs: rows {np.unique(d % nu)[:12]} cols {np.unique(d // nu)[:12]} "
                      f"max rel {np.max(np.abs(a[d] - b[d]) / np.maximum(np.abs(a[d]), 1e-300)):.3g}", flush=True)
            break
    F.close()


if __name__ == "__main__":
    main()
