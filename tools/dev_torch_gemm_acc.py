"""Dev: accuracy of the vendor fp64 GEMM (torch -> hipBLASLt/rocBLAS) against an extended-
precision host reference (is it a native fp64 GEMM?), and its rate on random data."""
import time
import numpy as np
import torch
torch.manual_seed(0)
for n, k in [(4096, 4096), (8192, 8192)]:
    a = torch.rand(n, k, dtype=torch.float64, device='cuda') - 0.5
    b = torch.rand(k, n, dtype=torch.float64, device='cuda') - 0.5
    c = a @ b
    torch.cuda.synchronize()
    reps = 5
    t = time.perf_counter()
    for _ in range(reps):
        c = a @ b
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / reps
    ah, bh, ch = a.cpu().numpy(), b.cpu().numpy(), c.cpu().numpy()
    rng = np.random.default_rng(1)
    errs, errs_naive = [], []
    for _ in range(200):
        i, j = rng.integers(0, n, 2)
        ex = np.dot(ah[i].astype(np.longdouble), bh[:, j].astype(np.longdouble))
        scale = np.dot(np.abs(ah[i]), np.abs(bh[:, j]))
        errs.append(float(abs(ch[i, j] - ex) / scale))
        nv = 0.0
        for q in range(0, k, 512):   # blocked fp64 dot (what a plain fp64 GEMM does)
            nv += float(np.dot(ah[i, q:q + 512], bh[q:q + 512, j]))
        errs_naive.append(float(abs(nv - ex) / scale))
    print(f"torch fp64 mm n={n} k={k}: {2*n*n*k/dt/1e12:.2f} TF/s; rel err max {max(errs):.2e} mean {np.mean(errs):.2e}"
          f" (numpy fp64 dot: max {max(errs_naive):.2e} mean {np.mean(errs_naive):.2e})", flush=True)
