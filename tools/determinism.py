"""Dev: bitwise determinism of refactor + solve at 3D Poisson N^3 (the pattern of
tests/test_gpu_fullsize.py::test_c3_poisson3d_128_refactor_steady_state), split into the solve
alone (same factors, solved twice) and refactor + solve (values refactored again).

    python tools/determinism.py 128        (env knobs such as SMLU_SOLVE_STEPS=1 per run)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sharedmemsparselu.jl_amd"))

import numpy as np  # noqa: E402


def main():
    import ctypes
    import torch
    import smlu
    import smlu._lib as C
    from smlu import matrices as mats
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    nosolve = len(sys.argv) > 2 and sys.argv[2] == "nosolve"   # factor hashes only, no solves
    A = mats.poisson3d(N)
    n = A.shape[0]
    F = smlu.ParallelSparseLU(A, device=0)
    dev = torch.device("cuda", 0)
    dpos = torch.from_numpy(mats.diag_positions(A)).to(dev)
    base = torch.from_numpy(np.ascontiguousarray(A.data)).to(dev)
    b = torch.from_numpy(np.random.default_rng(5).random(n)).to(dev)
    x = torch.empty_like(b)
    fn = C.lib().smlu_dev_front_hash
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    fn.restype = ctypes.c_int
    nsup = int(F.stat("nsuper"))

    def hashes():
        out = np.zeros(2 * nsup, np.uint64)
        assert fn(F._h, out.ctypes.data) == 0
        return out.reshape(nsup, 2)

    fr = F.fronts()
    first, parent, rowptr, fmode = fr["first"], fr["parent"], fr["rowptr"], fr["mode"]
    ns_, nu_ = np.diff(first), np.diff(rowptr)
    height = np.zeros(nsup, np.int64)
    for s in range(nsup):
        if parent[s] >= 0:
            height[parent[s]] = max(height[parent[s]], height[s] + 1)
    fv = C.lib().smlu_dev_front_values
    fv.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
    fv.restype = ctypes.c_int

    def values(s):
        M = ns_[s] + nu_[s]
        out = np.empty(M * ns_[s] + ns_[s] * nu_[s])
        assert fv(F._h, int(s), out.ctypes.data) == 0
        return out

    def diff_front(s0, va, vb):
        """Values of front s0 after refactoring va twice in a row vs after vb then va."""
        F.refactor_device(va)
        F.refactor_device(va)
        a1 = values(s0)
        F.refactor_device(vb)
        F.refactor_device(va)
        a2 = values(s0)
        M, ns, nu = int(ns_[s0] + nu_[s0]), int(ns_[s0]), int(nu_[s0])
        d = np.nonzero(a1 != a2)[0]
        print(f"   front {s0} (M {M}, ns {ns}, nu {nu}): {d.size} of {a1.size} entries depend on the previous values", flush=True)
        if d.size == 0:
            return
        lp = d[d < M * ns]
        up = d[d >= M * ns] - M * ns
        rows, cols = lp % M, lp // M
        reg = {"L11/U11": int(((rows < ns)).sum()), "L21": int((rows >= ns).sum()), "U12": int(up.size)}
        rel = np.abs(a1[d] - a2[d]) / np.maximum(np.abs(a1[d]), 1e-300)
        print(f"   regions {reg}; max rel diff {rel.max():.3g}; L-panel cols {np.unique(cols)[:12]} rows {np.unique(rows)[:12]}; "
              f"U12 rows {np.unique(up % max(ns, 1))[:12]} cols {np.unique(up // max(ns, 1))[:12]}", flush=True)

    hs = {}
    xs = []
    # first graph launch (the refactor right after create captures the graph) vs the second
    v = base.clone()
    v[dpos] += torch.from_numpy(np.random.default_rng(47).random(n)).to(dev)
    F.refactor_device(v)
    (None if nosolve else F.solve_device(x, b))
    xa = x.clone()
    F.refactor_device(v)
    (None if nosolve else F.solve_device(x, b))
    d = (x - xa).abs()
    print(f"v0 refactored twice in a row: max diff {d.max().item():.3g} differing {(d > 0).sum().item()}", flush=True)
    for r in range(5):
        v = base.clone()
        v[dpos] += torch.from_numpy(np.random.default_rng(47 + r).random(n)).to(dev)
        F.refactor_device(v)
        (None if nosolve else F.solve_device(x, b))
        hs[r] = hashes()
        x1 = x.clone()
        (None if nosolve else F.solve_device(x, b))
        d = (x - x1).abs().max().item()
        print(f"r={r} solve twice: max diff {d:.3g} bitwise {torch.equal(x, x1)} weak {F.stat('weak')} "
              f"timeouts {F.stat('sweep_timeouts')} refine_steps {F.stat('refine_steps')} repivots {F.stat('repivots')} "
              f"(last trigger node {F.stat('repivot_node')} info {F.stat('repivot_info')} mode {F.stat('repivot_node_mode')})",
              flush=True)
        xs.append((v, x.clone()))
    for r in (0, 1):
        v0, x0 = xs[r]
        F.refactor_device(v0)
        (None if nosolve else F.solve_device(x, b))
        d = (x - x0).abs()
        h = hashes()
        print(f"refactor v{r} again: max diff {d.max().item():.3g} differing {(d > 0).sum().item()} "
              f"bitwise {torch.equal(x, x0)}; repivots {F.stat('repivots')}; fronts with other factor values {(h[:, 0] != hs[r][:, 0]).sum()}, "
              f"other row perms {(h[:, 1] != hs[r][:, 1]).sum()}", flush=True)
        dv = np.nonzero(h[:, 0] != hs[r][:, 0])[0]
        if dv.size:
            order = dv[np.lexsort((dv, height[dv]))]
            print("   lowest differing fronts (s, height, mode, ns, nu):",
                  [(int(s), int(height[s]), int(fmode[s]), int(ns_[s]), int(nu_[s])) for s in order[:6]], flush=True)
    F.close()


if __name__ == "__main__":
    main()
