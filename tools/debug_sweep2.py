"""Dev: the single -> batch -> single sequence of tests/test_gpu_solve_sweep.py with errors against a CPU
reference for every vector."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "sharedmemsparselu.jl_amd"))


def main():
    import torch
    import scipy.sparse.linalg as spla
    import smlu
    from smlu import matrices as mats
    A = mats.poisson3d(40)
    n = A.shape[0]
    lu = spla.splu(A.tocsc())
    F = smlu.ParallelSparseLU(A)
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(9)
    b = torch.from_numpy(rng.random(n)).to(dev)
    x = torch.empty_like(b)
    F.solve_device(x, b)
    print("first", np.abs(x.cpu().numpy() - lu.solve(b.cpu().numpy())).max(), flush=True)
    for k in (2, 4, 8, 16):
        B = torch.from_numpy(rng.random((k, n))).to(dev)
        X = torch.empty_like(B)
        F.solve_multi_device(X, B)
        Bh = B.cpu().numpy()
        Xh = X.cpu().numpy()
        for j in range(k):
            F.solve_device(x, B[j].contiguous())
            xr = lu.solve(Bh[j])
            print(k, j, "batch err %.1e single err %.1e equal %s" % (np.abs(Xh[j] - xr).max(),
                  np.abs(x.cpu().numpy() - xr).max(), torch.equal(x, X[j])), flush=True)
    print("timeouts", F.stat("sweep_timeouts"))


if __name__ == "__main__":
    main()
