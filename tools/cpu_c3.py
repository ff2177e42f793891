"""The CPU baseline measured at the headline size (reproducibility of bench.py's
cpu_baseline).  On the GPU box's CPU share (OMP_NUM_THREADS, 16 for one GPU) it times the
multifrontal CPU port (oracle/mf.c, the GPU plan's assembly tree, partial pivoting, OpenMP):
3D Poisson 64^3 and 108^3 (bench.py's samples, 3 timed refactors each after an untimed one) and
the full 128^3 refactor (one untimed factorization, then one timed refactor, capped: the timed run
is skipped when the first took longer than --cap seconds).  Prints one JSON line.

    python tools/cpu_c3.py [--cap 200] > profiles/r04/cpu_c3.json
"""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "sharedmemsparselu.jl_amd"))

import numpy as np  # noqa: E402

import bench  # noqa: E402
import oracle as O  # noqa: E402
import smlu  # noqa: E402
from smlu import matrices as mats  # noqa: E402


def heartbeat():
    t0 = time.time()
    while True:
        time.sleep(30)
        print(f"[cpu_c3] alive {time.time() - t0:.0f} s", file=sys.stderr, flush=True)


def run(N, th, nrep, cap=None):
    A = mats.poisson3d(N)
    A.sort_indices()
    t0 = time.perf_counter()
    P = smlu.Plan(A)
    first, parent, rowptr, rows, p0 = P.fronts()
    fr = dict(first=first, parent=parent, rowptr=rowptr, rows=rows, p0=p0)
    mf = O.MultifrontalOracle(A, P.q(), fr, None, threads=th)
    t_plan = time.perf_counter() - t0
    t0 = time.perf_counter()
    st = mf.factor(A.data)
    t_first = time.perf_counter() - t0
    ts = []
    if cap is None or t_first <= cap:
        for _ in range(nrep):
            t0 = time.perf_counter()
            st = mf.factor(A.data)
            ts.append(time.perf_counter() - t0)
    mf.close()
    assert st == 0
    fl = P.stat("dense_flops")
    out = {"N": N, "threads": th, "plan_s": t_plan, "first_s": t_first, "timings": ts,
           "median_s": float(np.median(ts)) if ts else None, "dense_flops": fl, "nnzLU": P.stat("nnzLU"),
           "gflops": fl / (np.median(ts) if ts else t_first) / 1e9}
    print(f"[cpu_c3] {N}^3: first {t_first:.1f} s, timed {ts}", file=sys.stderr, flush=True)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cap", type=float, default=200.0)
    args = ap.parse_args()
    threading.Thread(target=heartbeat, daemon=True).start()
    th = bench.cpu_threads()
    res = {"threads": th, "nproc": os.cpu_count(), "runs": [run(64, th, 3), run(108, th, 3)]}
    full = run(128, th, 1, cap=args.cap)
    res["runs"].append(full)
    r108 = res["runs"][1]
    res["extrapolated_128_from_108_s"] = r108["median_s"] * full["dense_flops"] / r108["dense_flops"]
    res["measured_128_s"] = full["median_s"]
    print(json.dumps(res))


if __name__ == "__main__":
    main()
