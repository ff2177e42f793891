"""Dev helper: factor/solve a sweep of 3D Poisson sizes on the GPU and report timings."""
import sys, os, time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'sharedmemsparselu.jl_amd'))
import numpy as np
import smlu
from smlu import matrices as mats
for N in [int(a) for a in sys.argv[1:]] or [12, 16, 24, 32, 48, 64]:
    A = mats.poisson3d(N)
    t = time.time()
    try:
        F = smlu.ParallelSparseLU(A, profile=True)
    except Exception as e:
        print(N, 'FAILED', e, flush=True)
        break
    t1 = time.time() - t
    b = np.random.default_rng(0).random(A.shape[0]); x = np.empty_like(b)
    smlu.ldiv_(x, F, b)
    r = np.linalg.norm(A @ x - b) / np.linalg.norm(b)
    smlu.lu_(F, A)
    ks = {k: round(F.stat('ms_' + k), 2) for k in ['gemm', 'panel', 'trsm', 'small', 'assemble', 'memset']}
    print(N, 'create %.2fs' % t1, 'refactor %.1f ms' % F.stat('refactor_ms_last'), 'solve %.1f ms' % F.stat('solve_ms_last'),
          'resid %.2e' % r, 'nnzLU %.3g' % F.stat('nnzLU'), 'flops %.3g' % F.stat('dense_flops'), ks, flush=True)
    F.close()
