"""Solve timings at 3D Poisson N^3 on one GPU (dev measurement): one right-hand side (median of 7
solves), 8 right-hand sides batched (median of 3), each after a warm-up call, plus the refactor
time:

    python tools/solve_bench.py 128
"""
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
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    dev = torch.device("cuda:0")
    A = mats.poisson3d(N)
    F = smlu.ParallelSparseLU(A, device=0)
    n = A.shape[0]
    b = torch.from_numpy(np.random.default_rng(5).random(n)).to(dev)
    x = torch.empty_like(b)
    F.solve_device(x, b)
    torch.cuda.synchronize()
    t1 = []
    for _ in range(7):
        t0 = time.perf_counter()
        F.solve_device(x, b)
        torch.cuda.synchronize()
        t1.append((time.perf_counter() - t0) * 1e3)
    B8 = torch.from_numpy(np.random.default_rng(6).random((8, n))).to(dev)
    X8 = torch.empty_like(B8)
    F.solve_multi_device(X8, B8)
    torch.cuda.synchronize()
    t8 = []
    for _ in range(3):
        t0 = time.perf_counter()
        F.solve_multi_device(X8, B8)
        torch.cuda.synchronize()
        t8.append((time.perf_counter() - t0) * 1e3)
    F.solve_device(x, B8[3].contiguous())
    same = bool(torch.equal(x, X8[3]))
    xh, bh = x.cpu().numpy(), B8[3].cpu().numpy()
    res = float(np.abs(A @ xh - bh).max() / np.abs(bh).max())
    env = {k: v for k, v in os.environ.items() if k.startswith("SMLU_")}
    print(json.dumps({"N": N, "env": env, "solve_ms": float(np.median(t1)), "solve_ms_all": t1,
                      "solve8_ms": float(np.median(t8)), "solve8_ms_all": t8, "batch_col_bitwise": same,
                      "residual": res, "refactor_ms_last": F.stat("refactor_ms_last"),
                      "sweep_timeouts": F.stat("sweep_timeouts")}), flush=True)
    F.close()


if __name__ == "__main__":
    main()
