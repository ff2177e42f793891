"""Dev: per-refactor wall time at 128^3 in a few value-update patterns (in-place values, distinct
value tensors, profile on/off) -- the C5 steady-state diagnosis."""
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
    prof = len(sys.argv) > 2 and sys.argv[2] == "profile"
    dev = torch.device("cuda:0")
    A = mats.poisson3d(N)
    F = smlu.ParallelSparseLU(A, device=0, profile=prof)
    dpos = torch.from_numpy(mats.diag_positions(A)).to(dev)
    base = torch.from_numpy(np.ascontiguousarray(A.data)).to(dev)
    vals = torch.empty_like(base)
    g = torch.Generator(device=dev)
    for r in range(9):
        g.manual_seed(47 + r)
        vals.copy_(base)
        vals[dpos] += torch.rand(dpos.numel(), generator=g, device=dev, dtype=torch.float64)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        F.refactor_device(vals)
        t = (time.perf_counter() - t0) * 1e3
        print(f"in-place r={r} wall {t:.1f} ms lib {F.stat('refactor_ms_last'):.1f} ms dominant {F.stat('dominant')} "
              f"pivmode {F.stat('pivmode')} weak {F.stat('weak')} repivots {F.stat('repivots')} launches {F.stat('launches')}",
              flush=True)
    vs = []
    for r in range(3):
        v = base.clone()
        v[dpos] += torch.from_numpy(np.random.default_rng(100 + r).random(dpos.numel())).to(dev)
        vs.append(v)
    torch.cuda.synchronize()
    for r in range(6):
        t0 = time.perf_counter()
        F.refactor_device(vs[r % 3])
        t = (time.perf_counter() - t0) * 1e3
        print(f"distinct r={r} wall {t:.1f} ms lib {F.stat('refactor_ms_last'):.1f} ms", flush=True)


if __name__ == "__main__":
    main()
