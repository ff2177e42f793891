#!/usr/bin/env python3
"""One numeric factorization of the 3D Poisson N^3 matrix (the bench workload) and exit: the
target of the rocprofv3 PMC passes (tools/profile_pmc.sh), which need few dispatches."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sharedmemsparselu.jl_amd"))
import smlu  # noqa: E402
from smlu import matrices as mats  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 128
t0 = time.perf_counter()
F = smlu.ParallelSparseLU(mats.poisson3d(N))
print(f"N={N} factor+analysis {time.perf_counter() - t0:.1f}s gemm_launches={F.stat('gemm_launches'):.0f} "
      f"gemm_bytes={F.stat('gemm_bytes'):.6g} gemm_flops={F.stat('gemm_flops'):.6g}", flush=True)
F.close()
