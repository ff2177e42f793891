"""Dev: bitwise determinism of refactor + solve at 3D Poisson N^3 (the pattern of
tests/test_gpu_fullsize.py::test_c3_poisson3d_128_refactor_steady_state), split into the solve
alone (same factors, solved twice) and refactor + solve (values refactored again).

    python tools/determinism.py 128        (env knobs such as SMLU_SOLVE_STEPS=1 per run)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sharedmemsparselu.jl_amd"))

import numpy as np  # noqa: E402


def main():
    import torch
    import smlu
    from smlu import matrices as mats
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    A = mats.poisson3d(N)
    n = A.shape[0]
    F = smlu.ParallelSparseLU(A, device=0)
    dev = torch.device("cuda", 0)
    dpos = torch.from_numpy(mats.diag_positions(A)).to(dev)
    base = torch.from_numpy(np.ascontiguousarray(A.data)).to(dev)
    b = torch.from_numpy(np.random.default_rng(5).random(n)).to(dev)
    x = torch.empty_like(b)
    xs = []
    # first graph launch (the refactor right after create captures the graph) vs the second
    v = base.clone()
    v[dpos] += torch.from_numpy(np.random.default_rng(47).random(n)).to(dev)
    F.refactor_device(v)
    F.solve_device(x, b)
    xa = x.clone()
    F.refactor_device(v)
    F.solve_device(x, b)
    d = (x - xa).abs()
    print(f"v0 refactored twice in a row: max diff {d.max().item():.3g} differing {(d > 0).sum().item()}", flush=True)
    for r in range(5):
        v = base.clone()
        v[dpos] += torch.from_numpy(np.random.default_rng(47 + r).random(n)).to(dev)
        F.refactor_device(v)
        F.solve_device(x, b)
        x1 = x.clone()
        F.solve_device(x, b)
        d = (x - x1).abs().max().item()
        print(f"r={r} solve twice: max diff {d:.3g} bitwise {torch.equal(x, x1)} weak {F.stat('weak')} "
              f"timeouts {F.stat('sweep_timeouts')} refine_steps {F.stat('refine_steps')}", flush=True)
        xs.append((v, x.clone()))
    for r in (0, 1):
        v0, x0 = xs[r]
        F.refactor_device(v0)
        F.solve_device(x, b)
        d = (x - x0).abs()
        print(f"refactor v{r} again: max diff {d.max().item():.3g} differing {(d > 0).sum().item()} "
              f"bitwise {torch.equal(x, x0)}", flush=True)
    F.close()


if __name__ == "__main__":
    main()
