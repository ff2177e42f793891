"""Dev: sha1 of the exported factors (L, U values and the row permutation) and of device solves
(one and eight right-hand sides) of a few matrices, to check that a kernel change leaves the
factorization and the solves bitwise unchanged: run once per library (SMLU_LIB=...) and compare
the lines.

    SMLU_LIB=... python tools/factor_hash.py
"""
import hashlib
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "sharedmemsparselu.jl_amd"))


def main():
    import smlu
    from smlu import matrices as mats
    cases = []
    A = mats.perturb_diag(mats.poisson3d(64), 3)
    cases.append(("poisson3d64_dominant", A))
    B = mats.poisson3d(40).tocsc().copy()
    B.data = np.random.default_rng(5).standard_normal(B.nnz)
    cases.append(("poisson3d40_random_values", B))
    C = mats.poisson2d(256).tocsc().copy()
    C.data = C.data * (1.0 + 0.9 * np.random.default_rng(9).standard_normal(C.nnz))
    cases.append(("poisson2d256_weak_diagonal", C))
    for name, M in cases:
        F = smlu.ParallelSparseLU(M)
        h = hashlib.sha1()
        for arr in (F.L.data, F.U.data, np.asarray(F.p)):
            h.update(np.ascontiguousarray(arr).tobytes())
        # solutions: one right-hand side and a batch of eight (device solves)
        import torch
        n = M.shape[0]
        B = torch.from_numpy(np.random.default_rng(11).standard_normal((8, n))).cuda()
        X = torch.empty_like(B)
        F.solve_multi_device(X, B)
        x1 = torch.empty_like(B[0])
        F.solve_device(x1, B[0].contiguous())
        torch.cuda.synchronize()
        hs = hashlib.sha1(X.cpu().numpy().tobytes() + x1.cpu().numpy().tobytes()).hexdigest()[:16]
        print(name, h.hexdigest()[:16], "solves", hs, "repivots", F.stat("repivots"))
        F.close()


if __name__ == "__main__":
    main()
