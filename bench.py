#!/usr/bin/env python3
"""bench.py — numeric sparse-LU refactorization throughput on MI355X (BASELINE.json metric).

Step = one numeric refactorization (lu!(F, A): same pattern, new values) of the 3D 7-point
Poisson matrix (default 128^3, BASELINE config C3/C5), values already resident in HBM.
Prints ONE JSON line (rank 0).  Launch: ``python bench.py`` (1 GPU) or, for N GPUs,
``python -m torch.distributed.run --nproc-per-node N bench.py --gpus N``.

Multi-GPU (N > 1): ONE factorization split over the ranks — subtrees of the assembly tree per
rank, update blocks moved at exchange points over RCCL point-to-point ("scaling": "strong";
`--replicas` runs independent copies instead).  DESIGN.md §7.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "sharedmemsparselu.jl_amd"))

FP64_PEAK_TFLOPS = 78.6   # MI355X fp64 dense peak (vector == matrix on gfx950), AMD spec
HBM_PEAK_GBS = 8000.0     # MI355X HBM3E peak, MI355X_MICROARCH.md


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def cpu_baseline(N_cpu, ordering, grid_hint):
    """Oracle (scalar C port of the reference's fixed-pivot LU) on a bounded sample: the same
    workload family at N_cpu^3 with the same ordering algorithm, 1 core."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    import smlu
    from smlu import matrices as mats
    A = mats.poisson3d(N_cpu)
    P = smlu.Plan(A, grid=(N_cpu,) * 3 if grid_hint else None)
    q = P.q()
    Rs = O.rowscale(A)
    t0 = time.perf_counter()
    F = O.OracleLU(A, q, q, Rs)
    dt = time.perf_counter() - t0
    nnz = F.L.nnz + F.U.nnz - A.shape[0]
    one = {"value": nnz / dt, "unit": "nnz(L+U)/s", "cores": 1, "kind": "port",
           "sample": f"oracle fixed-pivot Gilbert-Peierls LU of 3D Poisson {N_cpu}^3 "
                     f"({ordering} order, nnz(L+U)={nnz}, upd={P.stat('upd'):.3g}) in {dt:.2f} s",
           "seconds": dt, "gflops": 2 * P.stat("upd") / dt / 1e9}
    # all host cores: the same factorization on C threads at once (the C oracle
    # runs without the GIL), aggregate throughput; C = the box's CPU share (16) or fewer
    from concurrent.futures import ThreadPoolExecutor
    C = max(1, min(16, os.cpu_count() or 1))
    t0 = time.perf_counter()
    with ThreadPoolExecutor(C) as ex:
        list(ex.map(lambda _: O.OracleLU(A, q, q, Rs), range(C)))
    dtc = time.perf_counter() - t0
    one["all_cores"] = {"value": C * nnz / dtc, "unit": "nnz(L+U)/s", "cores": C, "kind": "port",
                        "sample": f"{C} concurrent copies of the same factorization in {dtc:.2f} s"}
    return one


def max_over_ranks(x, device=None):
    """Max of a float over all ranks (identity when torch.distributed is not initialised)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device or "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def timed_region(step, steps, warmup, sync, device=None):
    """Contract of the driver: W untimed warmup steps, then EXACTLY `steps` steps bracketed by
    a barrier + device sync on both sides; returns the MAX wall time over ranks."""
    import torch.distributed as dist
    dist_on = dist.is_available() and dist.is_initialized()
    for r in range(warmup):
        step(r)
    if dist_on:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for r in range(steps):
        step(warmup + r)
    sync()
    if dist_on:
        dist.barrier()
    return max_over_ranks(time.perf_counter() - t0, device)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--side", "--n", dest="n", type=int, default=128,
                    help="grid side of the 3D Poisson workload")
    ap.add_argument("--ordering", default="nd", choices=["nd", "geometric"])
    ap.add_argument("--cpu-n", type=int, default=32, help="grid side of the CPU baseline sample")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-profile", action="store_true", help="skip per-kernel HIP events")
    ap.add_argument("--test-one-gpu", action="store_true",
                    help="rehearsal: all ranks on cuda:0, gloo transport (never for measurements)")
    ap.add_argument("--replicas", action="store_true",
                    help="N > 1: independent replicas instead of the partitioned factorization")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist
    if args.test_one_gpu:
        local = 0
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        if args.test_one_gpu:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
    else:
        torch.cuda.set_device(local)
    dev = torch.device(f"cuda:{local}")

    import smlu
    from smlu import matrices as mats
    N = args.n
    t0 = time.perf_counter()
    A = mats.poisson3d(N)
    n = A.shape[0]
    log(f"rank {rank}: generated 3D Poisson {N}^3 n={n} nnz={A.nnz} in {time.perf_counter()-t0:.1f}s")
    grid = (N, N, N) if args.ordering == "geometric" else None
    partitioned = world > 1 and not args.replicas
    t0 = time.perf_counter()
    if partitioned:   # one factorization split over the ranks (subtrees + RCCL exchanges)
        F = smlu.DistributedSparseLU(A, device=local, ordering=args.ordering,
                                     **({"grid": grid} if grid else {}))
    else:
        F = smlu.ParallelSparseLU(A, grid=grid, device=local, profile=not args.no_profile)
    t_create = time.perf_counter() - t0
    nnzLU = F.stat("nnzLU")
    log(f"rank {rank}: analysis {F.stat('analysis_ms')/1e3:.1f}s, create+first factor {t_create:.1f}s, "
        f"nnz(L+U)={nnzLU:.4g}, upd={F.stat('upd'):.4g}, launches={F.stat('launches'):.0f}"
        + (f", segments={F.nseg}" if partitioned else ""))

    # C5 inputs: same pattern, new values (diag += U(0,1) from default_rng(47+r)), uploaded to HBM
    dpos = torch.from_numpy(mats.diag_positions(A)).to(dev)
    base = torch.from_numpy(np.ascontiguousarray(A.data)).to(dev)
    vals = []
    for r in range(args.warmup + args.steps):
        v = base.clone()
        d = torch.from_numpy(np.random.default_rng(47 + r).random(n)).to(dev)
        v[dpos] += d
        vals.append(v)
    torch.cuda.synchronize()

    kinds = ["gemm", "gemmu", "gemmo", "gemm22", "panel", "trsm", "small", "assemble", "memset"]
    kind_ms = {k: 0.0 for k in kinds}

    def step(r):
        F.refactor_device(vals[r])
        if r >= args.warmup and not partitioned:
            for k in kinds:
                kind_ms[k] += F.stat("ms_" + k)
        log(f"rank {rank}: {'warmup' if r < args.warmup else 'step'} {r} refactor "
            f"{F.stat('refactor_ms_last'):.1f} ms")

    dt = timed_region(step, args.steps, args.warmup, torch.cuda.synchronize,
                      dev if world > 1 and not args.test_one_gpu else None)
    # one solve (reported, not the metric)
    b = torch.from_numpy(np.random.default_rng(5).random(n)).to(dev)   # same b on every rank
    x = torch.empty_like(b)
    F.solve_device(x, b)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    F.solve_device(x, b)
    torch.cuda.synchronize()
    solve_ms = (time.perf_counter() - t1) * 1e3
    # residual of that solve on the last refactored values (host SpMV)
    Al = A.copy()
    Al.data = vals[-1].cpu().numpy()
    xh, bh = x.cpu().numpy(), b.cpu().numpy()
    solve_residual = float(np.abs(Al @ xh - bh).max() / np.abs(bh).max())
    ms_per_step = dt / args.steps * 1e3

    if rank == 0:
        K = args.steps
        gemm_flops = F.stat("gemm_flops")
        ms_gemm = (kind_ms["gemm"] + kind_ms["gemmu"] + kind_ms["gemmo"] + kind_ms["gemm22"]) / K
        upd = F.stat("upd")
        dense_flops = F.stat("dense_flops")
        achieved = gemm_flops / (ms_gemm * 1e-3) / 1e12 if ms_gemm > 0 else None
        n_gemm = F.stat("gemm_launches")
        avg_us = ms_gemm * 1e3 / n_gemm if (n_gemm and ms_gemm > 0) else None
        traffic, traffic_src = None, "not collected"
        pmc = os.path.join(ROOT, "profiles", "r01", f"pmc_gemm_{N}.json")
        if os.path.exists(pmc):
            with open(pmc) as fh:
                pm = json.load(fh)
            traffic = pm.get("hbm_bytes_per_launch")
            traffic_src = os.path.relpath(pmc, ROOT)
        hbm_refactor = None
        if os.path.exists(pmc):
            hbm_refactor = pm.get("refactor_all_kernels", {}).get("hbm_bytes")
        nnzA = A.nnz
        # SURVEY §8(d) algorithmic bytes of the scatter/gather formulation, for reference
        bytes_sg = 12 * upd + 12 * nnzA + 12 * nnzLU + 16 * (n + 1)
        res = {
            "metric": "nnz(L+U)/s + achieved HBM GB/s, 3D Poisson 128³ numeric LU, 1/2/4/8 GPU",
            "value": nnzLU * (1 if partitioned else world) / (ms_per_step * 1e-3),
            "unit": "nnz(L+U)/s",
            "n_gpus": world,
            "steps": K,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "strong" if partitioned else "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {"workload": f"3D 7-point Poisson {N}^3 numeric refactorize (same pattern, "
                                   f"new diagonal values per step, values resident in HBM)",
                       "n": n, "nnzA": int(nnzA), "nnzLU": nnzLU, "upd": upd,
                       "dense_flops": dense_flops, "ordering": args.ordering,
                       "parallelism": (f"tree-partition{world} (proportional mapping, RCCL p2p)"
                                       if partitioned else f"replicas{world}" if world > 1 else "single")},
            "roofline": {"bound": "mfma", "kernel": "k_gemm128_mfma + k_gemm (fp64 Schur-complement updates)",
                         "achieved": achieved, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": (achieved / FP64_PEAK_TFLOPS) if achieved else None,
                         "traffic": traffic,
                         "launches_per_step": n_gemm, "avg_launch_us": avg_us,
                         "flops_per_launch": gemm_flops / n_gemm if n_gemm else None,
                         "algorithmic_bytes_per_launch": F.stat("gemm_bytes") / n_gemm if n_gemm else None,
                         "note": "fp64 MFMA (v_mfma_f64_16x16x4) 128x128 tiles for large launches, fp64 VALU "
                                 "64x64 tiles for small ones; peak = MI355X fp64 dense peak; "
                                 "achieved = GEMM flops per refactor / HIP-event time of the GEMM "
                                 "launches per refactor (graph-captured events on the launch "
                                 "stream); traffic = HBM bytes per launch from rocprofv3 PMC "
                                 "(FETCH_SIZE x2 + WRITE_SIZE, " + traffic_src + ")"},
            "kernel_ms_per_step": {k: v / K for k, v in kind_ms.items()},
            # per-kind HIP-event times exist for the single-GPU path only (partitioned: None)
            "gemm_split": ({"panel_tflops": (gemm_flops - F.stat("gemm22_flops")) / ((kind_ms["gemm"] + kind_ms["gemmu"] + kind_ms["gemmo"]) / K) / 1e9,
                            "f22_tflops": F.stat("gemm22_flops") / (kind_ms["gemm22"] / K) / 1e9,
                            "panel_gflop": (gemm_flops - F.stat("gemm22_flops")) / 1e9,
                            "f22_gflop": F.stat("gemm22_flops") / 1e9}
                           if ms_gemm > 0 and kind_ms["gemm22"] > 0 else None),
            "refactor_tflops": dense_flops / (ms_per_step * 1e-3) / 1e12,
            "scatter_gather_equiv_GBs": bytes_sg / (ms_per_step * 1e-3) / 1e9,
            # measured HBM traffic of a whole refactor (PMC FETCH_SIZE x2 + WRITE_SIZE over every
            # kernel, profiles/) over this run's time per refactor
            "achieved_hbm_GBs": (hbm_refactor / (ms_per_step * 1e-3) / 1e9) if hbm_refactor else None,
            "achieved_hbm_frac": (hbm_refactor / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS) if hbm_refactor else None,
            "solve_ms": solve_ms,
            "solve_residual": solve_residual,
            "create_s": t_create,
        }
        if not args.no_cpu and world == 1:
            log("cpu baseline ...")
            res["cpu_baseline"] = cpu_baseline(args.cpu_n, args.ordering, args.ordering == "geometric")
        print(json.dumps(res), flush=True)
    F.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
