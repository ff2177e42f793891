"""Multi-GPU partition rehearsed on one GPU: 2, 3 and 4 ranks (processes) share
cuda:0 and the library drives its transfers through the host-memory transport over gloo
(smlu/dist.py HostTransport); production runs use the library's RCCL transport with one GPU per
rank (same schedule, same packing, only the transfer calls differ).  Subtrees per rank, shared
top fronts as block-cyclic column partitions; the solution must match the single-GPU
factorization to rounding and solve A x = b to the reference tolerance on every rank."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _matrix(which):
    import scipy.sparse as sp
    from smlu import matrices as mats
    if which == "poisson":
        return sp.csc_matrix(mats.poisson3d(14))
    if which == "poisson_big":
        return sp.csc_matrix(mats.poisson3d(24))
    if which == "poisson40":
        return sp.csc_matrix(mats.poisson3d(40))
    return sp.csc_matrix(mats.random_dominant(3000, 0.003, seed=5))


def _values3(A):
    A3 = A.copy()
    A3.setdiag(A3.diagonal() * 2.0 + 1.0)
    import scipy.sparse as sp
    A3 = sp.csc_matrix(A3)
    A3.sort_indices()
    return A3.data


def _worker(rank, world, port, which, ob, q, transport="auto", gpu_per_rank=False):
    try:
        import scipy.sparse as sp
        import torch
        import torch.distributed as dist
        import smlu
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        if ob:
            os.environ["SMLU_OB"] = str(ob)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        dev = rank if gpu_per_rank else 0
        torch.cuda.set_device(dev)
        A = _matrix(which)
        n = A.shape[0]
        F = smlu.DistributedSparseLU(A, device=dev, transport=transport)
        b = np.random.default_rng(11).random(n)
        db = torch.from_numpy(b).cuda()
        dx = torch.empty_like(db)
        F.solve_device(dx, db)
        x1 = dx.cpu().numpy()
        # refactor with new values (same pattern) and solve again
        A2 = A.copy()
        A2.setdiag(A2.diagonal() + np.random.default_rng(3).random(n))
        A2 = sp.csc_matrix(A2)
        A2.sort_indices()
        F.refactor_device(torch.from_numpy(np.ascontiguousarray(A2.data)).cuda())
        F.solve_device(dx, db)
        x2 = dx.cpu().numpy()
        # lu! with host values on the partitioned handle (smlu_refactor, collective)
        F.refactor(_values3(A))
        F.solve_device(dx, db)
        x3 = dx.cpu().numpy()
        info = {k: F.stat(k) for k in ("shared_fronts", "owned_blocks", "comm_steps")}
        info["transport"] = F.transport
        q.put((rank, (x1, x3), x2, info, None))
        F.close()
        dist.destroy_process_group()
    except Exception:  # report instead of hanging the parent
        import traceback
        q.put((rank, None, None, None, traceback.format_exc()))


@pytest.mark.parametrize("world,which,ob", [(2, "poisson", 0), (4, "poisson", 0), (3, "random", 0),
                                            (2, "poisson_big", 128), (4, "poisson_big", 64),
                                            (8, "poisson40", 64)])
def test_dist_factor_solve_matches_single_gpu(world, which, ob):
    _run_and_compare(world, which, ob, "auto")


@pytest.mark.parametrize("world,which,ob", [(2, "poisson_big", 128), (4, "poisson_big", 64), (8, "poisson40", 64)])
def test_dist_device_memory_path_matches_single_gpu(world, which, ob):
    # the RCCL transport's calling convention (device buffers on the handle's stream, no host
    # staging in the library: exec_comm's device-memory branch, the addressing rccl_exchange /
    # rccl_bcast receive) with the bytes carried over gloo (smlu/dist.py DeviceStagedTransport)
    _run_and_compare(world, which, ob, "device")


def _run_and_compare(world, which, ob, transport):
    import scipy.sparse as sp
    import smlu
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, which, ob, q, transport)) for r in range(world)]
    for p in ps:
        p.start()
    # world 8: the rank count of the driver's 8-GPU scaling run (its partition and schedule)
    res = [q.get(timeout=420) for _ in ps]
    for p in ps:
        p.join(timeout=120)
    errs = [r[4] for r in res if r[4]]
    assert not errs, errs[0]
    for p in ps:
        assert p.exitcode == 0
    A = _matrix(which)
    n = A.shape[0]
    b = np.random.default_rng(11).random(n)
    A2 = A.copy()
    A2.setdiag(A2.diagonal() + np.random.default_rng(3).random(n))
    A2 = sp.csc_matrix(A2)
    F = smlu.ParallelSparseLU(A)
    xs1 = np.empty(n)
    smlu.ldiv_(xs1, F, b)
    smlu.lu_(F, A2)
    xs2 = np.empty(n)
    smlu.ldiv_(xs2, F, b)
    A3 = A.copy()
    A3.data = _values3(A)
    smlu.lu_(F, A3)
    xs3 = np.empty(n)
    smlu.ldiv_(xs3, F, b)
    F.close()
    # the partition really shares fronts between ranks and moves data
    assert max(r[3]["shared_fronts"] for r in res) >= 1
    assert all(r[3]["comm_steps"] >= 1 for r in res)
    if transport == "device":
        assert all(r[3]["transport"] == "device" for r in res)
    for rank, (x1, x3), x2, _, _ in res:
        # every rank holds the full solution
        assert np.allclose(x3, xs3, rtol=1e-11, atol=1e-13), (rank, np.abs(x3 - xs3).max())
        assert np.allclose(x1, xs1, rtol=1e-11, atol=1e-13), (rank, np.abs(x1 - xs1).max())
        assert np.allclose(x2, xs2, rtol=1e-11, atol=1e-13), (rank, np.abs(x2 - xs2).max())
        r1 = np.abs(A @ x1 - b).max() / np.abs(b).max()
        r2 = np.abs(A2 @ x2 - b).max() / np.abs(b).max()
        assert r1 < 1e-12 and r2 < 1e-12, (r1, r2)


def _weak_matrix():
    """Two 600-pivot dense blocks with tiny 64x64 diagonal tiles (weak diagonal-tile pivots),
    coupled only through a 64-column separator: under the natural order the assembly tree has
    two 600-column fronts below the separator front, so two ranks each factor one block and
    share the separator front."""
    import scipy.sparse as sp
    rng = np.random.default_rng(21)
    m, k = 600, 64
    n = 2 * m + k
    D = np.zeros((n, n))
    for b in (0, m):
        blk = rng.random((m, m))
        for b0 in range(0, m, 64):
            b1 = min(m, b0 + 64)
            blk[b0:b1, b0:b1] = 1e-2 * rng.random((b1 - b0, b1 - b0)) + 1e-2 * np.eye(b1 - b0)
        D[b:b + m, b:b + m] = blk
    # block 1 couples to separator rows/columns [0, 32), block 2 to [32, 64): the blocks' last
    # columns then do not nest into the separator (no supernode merge across it)
    h = k // 2
    for b, s0 in ((0, 0), (m, h)):
        D[2 * m + s0:2 * m + s0 + h, b:b + m] = rng.random((h, m))
        D[b:b + m, 2 * m + s0:2 * m + s0 + h] = rng.random((m, h))
    D[2 * m:, 2 * m:] = rng.random((k, k)) + k * np.eye(k)
    return sp.csc_matrix(D), D


def _weak_worker(rank, world, port, q):
    try:
        import torch
        import torch.distributed as dist
        import smlu
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        A, _ = _weak_matrix()
        n = A.shape[0]
        F = smlu.DistributedSparseLU(A, device=0, ordering="natural")
        b = torch.from_numpy(np.random.default_rng(4).random(n)).cuda()
        x = torch.empty_like(b)
        F.solve_device(x, b)
        q.put((rank, x.cpu().numpy(), F.weak, F.refine_steps, F.status, F.stat("shared_fronts"), None))
        F.close()
        dist.destroy_process_group()
    except Exception:
        import traceback
        q.put((rank, None, 0, 0, 0, 0, traceback.format_exc()))


def test_dist_weak_pivots_refine():
    # weak pivots on any rank are reduced over the partition (every rank sees them) and the
    # partitioned solve refines, as the single-GPU solve does
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_weak_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=240) for _ in ps]
    for p in ps:
        p.join(timeout=120)
    errs = [r[6] for r in res if r[6]]
    assert not errs, errs[0]
    _, D = _weak_matrix()
    b = np.random.default_rng(4).random(D.shape[0])
    xr = np.linalg.solve(D, b)
    ctol = max(1e-10, 8 * np.finfo(float).eps * np.linalg.cond(D))
    for rank, x, weak, steps, status, shared, _ in res:
        assert shared >= 1
        assert weak > 0 and steps >= 1, (rank, weak, status, steps)
        assert np.linalg.norm(x - xr) <= ctol * np.linalg.norm(xr), rank


def test_dist_rccl_transport_single_rank():
    # the library's built-in RCCL transport (the production multi-GPU path: librccl loaded by
    # libsmlu, unique id broadcast once over the control plane, communicator owned by the
    # handle) initialised and driven end to end on a one-rank partition -- two ranks cannot
    # share one GPU under RCCL ("duplicate GPU"), so the multi-rank exchanges are rehearsed
    # with the host transport above and run with RCCL on the 8-GPU node
    import smlu
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    p = ctx.Process(target=_worker, args=(0, 1, port, "poisson", 0, q, "rccl"))
    p.start()
    rank, x13, x2, info, err = q.get(timeout=240)
    p.join(timeout=120)
    assert err is None, err
    assert p.exitcode == 0
    assert info["transport"] == "rccl"
    A = _matrix("poisson")
    n = A.shape[0]
    b = np.random.default_rng(11).random(n)
    F = smlu.ParallelSparseLU(A)
    xs1 = np.empty(n)
    smlu.ldiv_(xs1, F, b)
    F.close()
    assert np.allclose(x13[0], xs1, rtol=1e-11, atol=1e-13)


def _gpu_count():
    import torch
    return torch.cuda.device_count()   # counts devices without initialising them


@pytest.mark.skipif(_gpu_count() < 2, reason="RCCL needs one GPU per rank (two or more GPUs)")
def test_dist_rccl_two_ranks_two_gpus():
    # the production multi-GPU path end to end: two processes, one GPU each, the library's own
    # RCCL communicator for every exchange and broadcast (xGMI), gloo only for the unique id
    import smlu
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, "poisson_big", 128, q, "rccl", True)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=240) for _ in ps], key=lambda r: r[0])
    for p in ps:
        p.join(timeout=120)
    errs = [r[4] for r in res if r[4]]
    assert not errs, errs[0]
    A = _matrix("poisson_big")
    n = A.shape[0]
    b = np.random.default_rng(11).random(n)
    F = smlu.ParallelSparseLU(A)
    xs = np.empty(n)
    smlu.ldiv_(xs, F, b)
    F.close()
    for rank, x13, x2, info, _ in res:
        assert info["transport"] == "rccl" and info["shared_fronts"] > 0
        assert np.allclose(x13[0], xs, rtol=1e-11, atol=1e-13), rank


def _spin_worker(rank, world, port, which, ob, q):
    # two partitioned handles on the same matrix: the default bounded waits, and SMLU_SWEEP_SPIN=0
    # (every sync-free sweep wait reports a timeout on every rank) -> the solve must be re-run on
    # the per-block schedule with the remapped comm segments and give the same x bitwise
    try:
        import torch
        import torch.distributed as dist
        import smlu
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        if ob:
            os.environ["SMLU_OB"] = str(ob)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        A = _matrix(which)
        n = A.shape[0]
        db = torch.from_numpy(np.random.default_rng(11).random(n)).cuda()
        F = smlu.DistributedSparseLU(A, device=0)
        dx = torch.empty_like(db)
        F.solve_device(dx, db)
        x_ref = dx.cpu().numpy()
        t_ref = F.stat("sweep_timeouts")
        sweeps = F.stat("solve_sweeps")
        F.close()
        os.environ["SMLU_SWEEP_SPIN"] = "0"
        G = smlu.DistributedSparseLU(A, device=0)
        dx2 = torch.empty_like(db)
        G.solve_device(dx2, db)
        x_spin = dx2.cpu().numpy()
        t_spin = G.stat("sweep_timeouts")
        sweeps_all = G.stat("solve_sweeps")
        G.close()
        q.put((rank, x_ref, x_spin, (t_ref, t_spin, sweeps, sweeps_all), None))
        dist.destroy_process_group()
    except Exception:
        import traceback
        q.put((rank, None, None, None, traceback.format_exc()))


@pytest.mark.parametrize("world,which,ob", [(2, "poisson_big", 128), (4, "poisson40", 128)])
def test_dist_forced_sweep_timeout_reruns_per_block(world, which, ob):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_spin_worker, args=(r, world, port, which, ob, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=300) for _ in ps]
    for p in ps:
        p.join(timeout=120)
    errs = [r[4] for r in res if r[4]]
    assert not errs, errs[0]
    assert any(r[3][2] > 0 for r in res), "no rank runs a sync-free sweep: the test would prove nothing"
    A = _matrix(which)
    b = np.random.default_rng(11).random(A.shape[0])
    for rank, x_ref, x_spin, (t_ref, t_spin, sweeps, _), _ in res:
        assert t_ref == 0, rank
        assert t_spin > 0, (rank, t_spin, sweeps)   # the allreduced flag: every rank re-ran
        assert np.array_equal(x_ref, x_spin), (rank, np.abs(x_ref - x_spin).max())
        assert np.abs(A @ x_spin - b).max() / np.abs(b).max() < 1e-12
