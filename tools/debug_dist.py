"""Dev: run the partitioned factorization + solve with W ranks sharing cuda:0 (gloo) and report,
per front (in elimination order), the max error of x against the single-GPU solve."""
import os, sys, socket
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "sharedmemsparselu.jl_amd"))
import numpy as np
import torch.multiprocessing as mp


def port():
    s = socket.socket(); s.bind(("127.0.0.1", 0)); p = s.getsockname()[1]; s.close(); return p


def mat(N):
    import scipy.sparse as sp
    from smlu import matrices as mats
    return sp.csc_matrix(mats.poisson3d(N))


def worker(rank, world, pt, N, q):
    try:
        import torch, torch.distributed as dist, smlu
        os.environ["MASTER_ADDR"] = "127.0.0.1"; os.environ["MASTER_PORT"] = str(pt)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        A = mat(N)
        F = smlu.DistributedSparseLU(A, device=0)
        b = torch.from_numpy(np.random.default_rng(11).random(A.shape[0])).cuda()
        x = torch.empty_like(b)
        F.solve_device(x, b)
        q.put((rank, x.cpu().numpy(), None))
        F.close(); dist.destroy_process_group()
    except Exception:
        import traceback; q.put((rank, None, traceback.format_exc()))


if __name__ == "__main__":
    world = int(sys.argv[1]); N = int(sys.argv[2])
    import smlu
    ctx = mp.get_context("spawn"); q = ctx.Queue(); pt = port()
    ps = [ctx.Process(target=worker, args=(r, world, pt, N, q)) for r in range(world)]
    [p.start() for p in ps]
    res = sorted([q.get(timeout=200) for _ in ps], key=lambda r: r[0])
    [p.join(timeout=60) for p in ps]
    for r in res:
        if r[2]: print(r[2])
    A = mat(N); n = A.shape[0]
    b = np.random.default_rng(11).random(n)
    F = smlu.ParallelSparseLU(A); xs = np.empty(n); smlu.ldiv_(xs, F, b)
    P = smlu.Plan(A); qq = P.q(); first, parent, level = P.supernodes(); owner, nsh = P.partition(world)
    print("shared fronts", nsh, [int(s) for s in np.where(owner < 0)[0]])
    for rank, x, err in res:
        if x is None: continue
        d = np.abs(x - xs)[qq]
        bad = []
        for s in range(len(parent)):
            e = d[first[s]:first[s + 1]].max()
            if e > 1e-10: bad.append((s, int(owner[s]), int(level[s]), float(e)))
        print("rank", rank, "max err", d.max(), "bad fronts", len(bad), bad[:12])
