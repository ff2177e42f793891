"""Dev: is the spurious re-pivoting refactor of in-place value updates (C5) a property of the values
or of the handle's history?  In-place updates as tools/c5_steady.py; on the first re-pivot the
values are checked on the host and factored again by the same handle and by a fresh one."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sharedmemsparselu.jl_amd"))

import numpy as np  # noqa: E402
import scipy.sparse as sp  # noqa: E402


def dominant(A):
    A = sp.csc_matrix(A)
    d = np.abs(A.diagonal())
    r = np.asarray(abs(A).sum(axis=1)).ravel() - d
    c = np.asarray(abs(A).sum(axis=0)).ravel() - d
    return bool((d >= r).all()), bool((d >= c).all()), float((d - r).min()), float((d - c).min())


def main():
    import torch
    import smlu
    from smlu import matrices as mats
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    dev = torch.device("cuda:0")
    A = mats.poisson3d(N)
    F = smlu.ParallelSparseLU(A, device=0)
    dpos = torch.from_numpy(mats.diag_positions(A)).to(dev)
    base = torch.from_numpy(np.ascontiguousarray(A.data)).to(dev)
    vals = torch.empty_like(base)
    g = torch.Generator(device=dev)
    print("pointers: vals", hex(vals.data_ptr()), "base", hex(base.data_ptr()), "dpos", hex(dpos.data_ptr()), flush=True)
    for r in range(12):
        g.manual_seed(47 + r)
        vals.copy_(base)
        vals[dpos] += torch.rand(dpos.numel(), generator=g, device=dev, dtype=torch.float64)
        torch.cuda.synchronize()
        rp0 = F.stat("repivots")
        F.refactor_device(vals)
        print(f"r={r} repivots {F.stat('repivots')} pivmode {F.stat('pivmode')} weak {F.stat('weak')} "
              f"trigger node {F.stat('repivot_node')} info {F.stat('repivot_info')} mode {F.stat('repivot_node_mode')} "
              f"ns {F.stat('repivot_node_ns')} nu {F.stat('repivot_node_nu')} g {F.stat('repivot_growth'):.3g} "
              f"growth {F.stat('growth_max'):.3g}", flush=True)
        if F.stat("repivots") > rp0:
            vh = vals.cpu().numpy()
            A2 = A.copy()
            A2.data = vh.copy()
            print("  host dominance (rows, cols, min margins):", dominant(A2), "finite", np.isfinite(vh).all(),
                  "diag min/max", A2.diagonal().min(), A2.diagonal().max(), flush=True)
            F.refactor_device(vals)
            print(f"  same handle again: repivots {F.stat('repivots')} pivmode {F.stat('pivmode')}", flush=True)
            G = smlu.ParallelSparseLU(A2, device=0)
            print(f"  fresh handle: repivots {G.stat('repivots')} pivmode {G.stat('pivmode')} weak {G.stat('weak')}", flush=True)
            G2 = smlu.ParallelSparseLU(A, device=0)
            G2.refactor_device(torch.from_numpy(vh).to(dev))
            print(f"  fresh handle + refactor_device: repivots {G2.stat('repivots')} weak {G2.stat('weak')}", flush=True)
            G.close()
            G2.close()
            break


if __name__ == "__main__":
    main()
