#!/usr/bin/env python3
"""Host-only: the analysis time and peak host RSS of the C3 / C4 plans, the calibrated projection of
the partitioned factorization at 1/2/4/8 ranks (smlu_plan_project: level-batched fronts, 80 us per
64-column panel step, 0.32 ms per level, 52 TFLOP/s of dense front work -- DESIGN.md §7) and the
device memory per rank (smlu_plan_rank_memory).  Usage: python tools/partition_projection.py
[sides ...] > profiles/<round>/partition_projection.txt"""
import os
import resource
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sharedmemsparselu.jl_amd"))

import smlu  # noqa: E402
from smlu import matrices as mats  # noqa: E402


def rss_mb():
    return resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1024.0


def main():
    sides = [int(a) for a in sys.argv[1:]] or [128, 256]
    threads = os.cpu_count()
    print(f"# smlu_plan_project (calibrated: 52 TFLOP/s, 100 GB/s links, 20 us latency, 80 us per panel "
          f"step, 0.32 ms per level), graph-ND ordering; host threads {threads}")
    phases = ["input", "graph", "order", "etree", "colcount", "rowstruct", "relax", "levels", "layout", "amap"]
    for N in sides:
        t0 = time.perf_counter()
        A = mats.poisson3d(N)
        tg = time.perf_counter() - t0
        r0 = rss_mb()
        t0 = time.perf_counter()
        P = smlu.Plan(A)
        ta = time.perf_counter() - t0
        r1 = rss_mb()
        print(f"## {N}^3: n {A.shape[0]} nnz(A) {A.nnz}  nnz(L+U) {P.stat('nnzLU'):.4g}  dense flops "
              f"{P.stat('dense_flops'):.4g}  levels {P.stat('nlevels'):.0f}")
        print(f"analysis {ta:.1f} s (matrix generation {tg:.1f} s); peak host RSS {r1:.0f} MB "
              f"(after generating A: {r0:.0f} MB)")
        print("phases ms: " + " ".join(f"{nm}={P.stat('phase_ms%d' % i):.0f}" for i, nm in enumerate(phases)))
        print("# nparts projected_s one_gpu_s speedup  max_store_GB max_scratch_GB")
        for k in (1, 2, 4, 8):
            t, t1 = P.project(k)
            mem = [P.rank_memory(k, r) for r in range(k)]
            print(f"{k} {t:.4f} {t1:.4f} {t1 / t:.2f}  {max(m[0] for m in mem) / 1e9:.1f} "
                  f"{max(m[1] for m in mem) / 1e9:.1f}", flush=True)
        del P, A


if __name__ == "__main__":
    main()
