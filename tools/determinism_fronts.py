"""Dev: localise a non-reproducible factorization.  The same values (v1) are refactored again after
other values (v2) in between, several times; each time the per-front hashes of the factor values
and row permutations (smlu_dev_front_hash) are compared with the first run's, and the differing
fronts nearest the leaves are listed with their height in the tree, mode, ns and nu.

    python tools/determinism_fronts.py 128 [trials]
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
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    trials = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    A = mats.poisson3d(N)
    n = A.shape[0]
    F = smlu.ParallelSparseLU(A, device=0)
    fr = F.fronts()
    first, parent, rowptr, mode = fr["first"], fr["parent"], fr["rowptr"], fr["mode"]
    ns_ = np.diff(first)
    nu_ = np.diff(rowptr)
    nsup = ns_.size
    height = np.zeros(nsup, np.int64)   # children come before parents (postorder)
    for s in range(nsup):
        p = parent[s]
        if p >= 0:
            height[p] = max(height[p], height[s] + 1)
    fn = C.lib().smlu_dev_front_hash
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    fn.restype = ctypes.c_int

    def hashes():
        out = np.zeros(2 * nsup, np.uint64)
        assert fn(F._h, out.ctypes.data) == 0
        return out.reshape(nsup, 2)

    dev = torch.device("cuda", 0)
    dpos = torch.from_numpy(mats.diag_positions(A)).to(dev)
    base = torch.from_numpy(np.ascontiguousarray(A.data)).to(dev)
    vs = []
    for seed in (47, 48):
        v = base.clone()
        v[dpos] += torch.from_numpy(np.random.default_rng(seed).random(n)).to(dev)
        vs.append(v)
    b = torch.from_numpy(np.random.default_rng(5).random(n)).to(dev)
    x = torch.empty_like(b)
    solve = len(sys.argv) > 3 and sys.argv[3] == "solve"   # a solve after every refactor

    def refactor(v):
        F.refactor_device(v)
        if solve:
            h1 = hashes()
            F.solve_device(x, b)
            h2 = hashes()
            if not np.array_equal(h1, h2):
                print("   the solve changed factor values of", int((h1[:, 0] != h2[:, 0]).sum()), "fronts", flush=True)
            return x.clone()
        return None

    x0 = refactor(vs[0])
    H0 = hashes()
    for t in range(trials):
        refactor(vs[1])
        xt = refactor(vs[0])
        H = hashes()
        if solve:
            d = (xt - x0).abs()
            print(f"trial {t}: solution differs in {(d > 0).sum().item()} entries (max {d.max().item():.3g})", flush=True)
        dv = np.nonzero(H[:, 0] != H0[:, 0])[0]
        dp = np.nonzero(H[:, 1] != H0[:, 1])[0]
        print(f"trial {t}: fronts with different values {dv.size}, different row permutations {dp.size}", flush=True)
        if dv.size:
            order = dv[np.lexsort((dv, height[dv]))]
            for s in order[:8]:
                print(f"   front {s}: height {height[s]} mode {mode[s]} ns {ns_[s]} nu {nu_[s]} "
                      f"perm differs {bool(H[s, 1] != H0[s, 1])} parent {parent[s]}", flush=True)
    F.close()


if __name__ == "__main__":
    main()
