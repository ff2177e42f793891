"""C2 (2D 5-point Poisson 512^2) refactor + solve on one GPU (dev; the profile of the latency-bound
config): create, 20 refactors with new diagonal values resident in HBM, 20 solves; prints the
median times.  Under rocprofv3 --kernel-trace, tools/ktrace_summary.py summarises the last refactor
and solve."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sharedmemsparselu.jl_amd"))

import numpy as np  # noqa: E402


def main():
    import torch
    import smlu
    from smlu import matrices as mats
    dev = torch.device("cuda:0")
    A = mats.poisson2d(512)
    n = A.shape[0]
    F = smlu.ParallelSparseLU(A, device=0)
    dpos = torch.from_numpy(mats.diag_positions(A)).to(dev)
    base = torch.from_numpy(np.ascontiguousarray(A.data)).to(dev)
    vals = []
    for r in range(4):
        v = base.clone()
        v[dpos] += torch.from_numpy(np.random.default_rng(100 + r).random(n)).to(dev)
        vals.append(v)
    b = torch.from_numpy(np.random.default_rng(5).random(n)).to(dev)
    x = torch.empty_like(b)
    tr, ts = [], []
    for r in range(20):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        F.refactor_device(vals[r % 4])
        torch.cuda.synchronize()
        tr.append((time.perf_counter() - t0) * 1e3)
        t0 = time.perf_counter()
        F.solve_device(x, b)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    print(json.dumps({"config": "C2 2D Poisson 512^2", "n": n, "nnzLU": F.stat("nnzLU"), "launches": F.stat("launches"),
                      "nlevels": F.stat("nlevels"), "refactor_ms_median": float(np.median(tr[2:])),
                      "solve_ms_median": float(np.median(ts[2:])), "refactor_ms": tr, "solve_ms": ts}))


if __name__ == "__main__":
    main()
