"""Solve timing on the 3D Poisson workload: one right-hand side (smlu_solve_device) and batches
of 8 / 16 (smlu_solve_multi_device), median of several device-resident runs.  Run under
`rocprofv3 --kernel-trace --stats` to split the time over the solve kernels.

    python tools/solve_timing.py [--side 128] [--reps 5]
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "sharedmemsparselu.jl_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--side", type=int, default=128)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import torch
    import smlu
    from smlu import matrices as mats
    A = mats.poisson3d(args.side)
    n = A.shape[0]
    F = smlu.ParallelSparseLU(A, profile=False)
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(3)
    out = {"side": args.side, "n": n}

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(args.reps):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        return float(np.median(ts))

    b = torch.from_numpy(rng.random(n)).to(dev)
    x = torch.empty_like(b)
    out["ms_1"] = timed(lambda: F.solve_device(x, b))
    for k in (2, 4, 8, 16, 32):
        B = torch.from_numpy(rng.random((k, n))).to(dev)
        X = torch.empty_like(B)
        out[f"ms_{k}"] = timed(lambda: F.solve_multi_device(X, B))
        # columns agree with single-vector solves
        F.solve_device(x, B[k - 1].contiguous())
        assert torch.equal(x, X[k - 1]), k
    out["ratio_8"] = out["ms_8"] / out["ms_1"]
    print(out, flush=True)


if __name__ == "__main__":
    main()
