"""Dev check of the sync-free solve sweep: single and batched solves against a CPU reference,
repeated, with the sweep and with the per-block schedule (SMLU_SOLVE_STEPS=1)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "sharedmemsparselu.jl_amd"))


def main():
    import torch
    import scipy.sparse.linalg as spla
    import smlu
    from smlu import matrices as mats
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    A = mats.poisson3d(N)
    n = A.shape[0]
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(9)
    Bh = rng.random((16, n))
    lu = spla.splu(A.tocsc())
    Xr = np.stack([lu.solve(Bh[j]) for j in range(16)])
    for steps in ("0", "1"):
        os.environ["SMLU_SOLVE_STEPS"] = steps
        F = smlu.ParallelSparseLU(A)
        print("steps", steps, "sweeps", F.stat("solve_sweeps"), flush=True)
        x = torch.empty(n, dtype=torch.float64, device=dev)
        for rep in range(3):
            errs = []
            for j in range(4):
                F.solve_device(x, torch.from_numpy(Bh[j].copy()).to(dev))
                errs.append(np.abs(x.cpu().numpy() - Xr[j]).max())
            print(" single rep", rep, ["%.1e" % e for e in errs], "timeouts", F.stat("sweep_timeouts"), flush=True)
        for k in (2, 4, 8, 16):
            B = torch.from_numpy(Bh[:k].copy()).to(dev)
            X = torch.empty_like(B)
            F.solve_multi_device(X, B)
            Xh = X.cpu().numpy()
            print(" batch", k, ["%.1e" % np.abs(Xh[j] - Xr[j]).max() for j in range(k)], flush=True)
        F.close()


if __name__ == "__main__":
    main()
