"""BASELINE config C5 at its stated size: 1000 numeric refactorizations of the 3D Poisson 128^3
matrix (same pattern, new values every time: diag += U(0,1) drawn on the device from a generator
seeded 47 + r), values resident in HBM.  Records the per-refactor wall time (each smlu_refactor_device
call returns after its stream synchronisation), device memory before and after, and the residual of
a solve after the last refactor.  Prints progress every 50 refactors and one JSON line at the end.

    python tools/c5_steady.py [--n 128] [--reps 1000] > profiles/r04/c5_128_1000.json
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sharedmemsparselu.jl_amd"))

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=128)
    ap.add_argument("--reps", type=int, default=1000)
    args = ap.parse_args()
    import torch
    import smlu
    from smlu import matrices as mats
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    free0, total = torch.cuda.mem_get_info()
    A = mats.poisson3d(args.n)
    nnz = A.nnz
    t0 = time.perf_counter()
    F = smlu.ParallelSparseLU(A, device=0)
    create_s = time.perf_counter() - t0
    free1, _ = torch.cuda.mem_get_info()
    dpos = torch.from_numpy(mats.diag_positions(A)).to(dev)
    base = torch.from_numpy(np.ascontiguousarray(A.data)).to(dev)
    vals = torch.empty_like(base)
    g = torch.Generator(device=dev)
    times = []
    t_start = time.perf_counter()
    for r in range(args.reps):
        g.manual_seed(47 + r)
        vals.copy_(base)
        vals[dpos] += torch.rand(dpos.numel(), generator=g, device=dev, dtype=torch.float64)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        F.refactor_device(vals)
        times.append(time.perf_counter() - t0)
        if (r + 1) % 50 == 0:
            print(f"[c5] {r + 1} refactors, last {times[-1] * 1e3:.1f} ms, median {np.median(times) * 1e3:.1f} ms",
                  file=sys.stderr, flush=True)
    wall = time.perf_counter() - t_start
    free2, _ = torch.cuda.mem_get_info()
    b = torch.from_numpy(np.random.default_rng(5).random(A.shape[0])).to(dev)
    x = torch.empty_like(b)
    F.solve_device(x, b)
    Al = A.copy()
    Al.data = vals.cpu().numpy()
    xh, bh = x.cpu().numpy(), b.cpu().numpy()
    resid = float(np.abs(Al @ xh - bh).max() / np.abs(bh).max())
    t = np.array(times) * 1e3
    nnzLU = F.stat("nnzLU")
    out = {"config": f"C5: 3D Poisson {args.n}^3, {args.reps} numeric refactors, new values each (diag += U(0,1), "
                     f"device generator seeded 47+r), values resident in HBM",
           "n": A.shape[0], "nnzA": nnz, "nnzLU": nnzLU, "create_s": create_s, "refactors": args.reps,
           "wall_s_incl_value_generation": wall,
           "refactor_ms": {"mean": float(t.mean()), "median": float(np.median(t)), "min": float(t.min()),
                           "max": float(t.max()), "p05": float(np.percentile(t, 5)), "p95": float(np.percentile(t, 95)),
                           "std": float(t.std()), "first10": [float(v) for v in t[:10]], "last10": [float(v) for v in t[-10:]]},
           "steady_state_nnzLU_per_s": nnzLU / (float(np.median(t)) * 1e-3),
           "device_mem_GB": {"total": total / 1e9, "used_before_create": (total - free0) / 1e9,
                             "used_after_create": (total - free1) / 1e9, "used_after_last_refactor": (total - free2) / 1e9},
           "residual_after_last": resid, "weak_pivots_last": F.stat("weak"), "repivots": F.stat("repivots")}
    F.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
