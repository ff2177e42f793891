"""Dev: one dense diagonally-dominant front (n x n) -> blocked path; timing per refactor."""
import sys, os, time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'sharedmemsparselu.jl_amd'))
import numpy as np, scipy.sparse as sp
import smlu
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
rng = np.random.default_rng(0)
D = rng.random((n, n)); D += np.diag(D.sum(axis=1) + 1)
A = sp.csc_matrix(D)
F = smlu.ParallelSparseLU(A, profile=True)
for r in range(3):
    smlu.lu_(F, A)
    ks = {k: round(F.stat('ms_' + k), 2) for k in ['gemm', 'gemm22', 'panel', 'trsm', 'small', 'assemble', 'memset']}
    print(n, 'refactor %.2f ms' % F.stat('refactor_ms_last'), ks, 'launches', F.stat('launches'), flush=True)
b = rng.random(n); x = np.empty(n); smlu.ldiv_(x, F, b)
print('resid', np.linalg.norm(D @ x - b) / np.linalg.norm(b))
