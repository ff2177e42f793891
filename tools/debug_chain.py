"""Dev: one solve per size on the 3D Poisson workload with the current solve path, printing
time and residual per size (flushes after every line).  python tools/debug_chain.py 32 64 96"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "sharedmemsparselu.jl_amd"))


def main():
    import smlu
    from smlu import matrices as mats
    for side in map(int, sys.argv[1:]):
        A = mats.poisson3d(side)
        t0 = time.time()
        F = smlu.ParallelSparseLU(A, profile=False)
        print(f"side {side}: create {time.time() - t0:.2f} s", flush=True)
        b = np.random.default_rng(1).standard_normal(A.shape[0])
        for k in range(3):
            t0 = time.time()
            try:
                x = smlu.ldiv_(np.empty_like(b), F, b)
            except Exception as e:
                print(f"  solve {k}: error {e}", flush=True)
                return 1
            dt = time.time() - t0
            r = np.abs(A @ x - b).max() / np.abs(b).max()
            print(f"  solve {k}: {dt * 1e3:.2f} ms residual {r:.2e}", flush=True)
        F.close() if hasattr(F, "close") else None
    return 0


if __name__ == "__main__":
    sys.exit(main())
