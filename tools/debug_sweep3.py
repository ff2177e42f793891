"""Dev: bisect the single-after-batch sweep failure over sweep modes / graph use (one subprocess each)."""
import os
import subprocess
import sys

CODE = r'''
import os, sys
import numpy as np
sys.path.insert(0, "sharedmemsparselu.jl_amd")
import torch, scipy.sparse.linalg as spla, smlu
from smlu import matrices as mats
A = mats.poisson3d(40); n = A.shape[0]; lu = spla.splu(A.tocsc())
F = smlu.ParallelSparseLU(A); dev = torch.device("cuda:0"); rng = np.random.default_rng(9)
b = torch.from_numpy(rng.random(n)).to(dev); x = torch.empty_like(b)
F.solve_device(x, b)
out = ["first %.0e" % np.abs(x.cpu().numpy() - lu.solve(b.cpu().numpy())).max()]
B = torch.from_numpy(rng.random((2, n))).to(dev); X = torch.empty_like(B)
F.solve_multi_device(X, B)
out.append("batch %.0e" % np.abs(X[1].cpu().numpy() - lu.solve(B[1].cpu().numpy())).max())
for j in range(2):
    F.solve_device(x, B[j].contiguous())
    out.append("single%d %.0e" % (j, np.abs(x.cpu().numpy() - lu.solve(B[j].cpu().numpy())).max()))
out.append("timeouts %d" % F.stat("sweep_timeouts"))
print(" ".join(out), flush=True)
'''

for env in ({"SMLU_SWEEP_MODE": "8"}, {"SMLU_SWEEP_MODE": "9"}, {"SMLU_SWEEP_MODE": "11"},
            {"SMLU_SWEEP_MODE": "8", "SMLU_NO_GRAPH": "1"}):
    e = dict(os.environ, **env)
    r = subprocess.run([sys.executable, "-c", CODE], env=e, capture_output=True, text=True, timeout=120)
    print(env, r.stdout.strip(), r.returncode, r.stderr.strip()[-300:] if r.returncode else "", flush=True)
