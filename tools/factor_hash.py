"""Dev: sha1 of the exported factors (L, U values and the row permutation) of a few matrices, to
check that a kernel change leaves the factorization bitwise unchanged: run once per library
(SMLU_LIB=...) and compare the lines.

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
        print(name, h.hexdigest()[:16], "repivots", F.stat("repivots") if hasattr(F, "stat") else "")
        F.close()


if __name__ == "__main__":
    main()
