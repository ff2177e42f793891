"""Dev: vendor fp64 GEMM rate (torch -> hipBLASLt/rocBLAS) as a ceiling reference."""
import torch, time
for n, k in [(4096, 4096), (8192, 8192), (16384, 64), (16384, 256), (12000, 6000)]:
    a = torch.rand(n, k, dtype=torch.float64, device='cuda'); b = torch.rand(k, n, dtype=torch.float64, device='cuda')
    c = torch.rand(n, n, dtype=torch.float64, device='cuda')
    c.addmm_(a, b, alpha=-1); torch.cuda.synchronize()
    reps = 5
    t = time.perf_counter()
    for _ in range(reps): c.addmm_(a, b, alpha=-1)
    torch.cuda.synchronize(); dt = (time.perf_counter() - t) / reps
    print(f"torch fp64 addmm m=n={n} k={k}: {2*n*n*k/dt/1e12:.2f} TF/s", flush=True)
