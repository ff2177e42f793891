"""Per-dispatch GEMM efficiency of one eager factorization (dev).

Joins a rocprofv3 kernel trace of tools/pmc_factor.py (run with SMLU_NO_GRAPH=1 and
SMLU_DUMP_SCHEDULE=<csv>) with the library's schedule dump: the k_gemm* dispatches appear in
schedule order.  Prints TFLOP/s by launch kind, by tile count (wave quantisation: 512 tile
slots = 256 CUs x 2 workgroups) and by k.
Usage: python tools/gemm_dispatch_report.py <kernel_trace.csv> <schedule.csv>
"""
import csv
import sys
from collections import defaultdict

tr = list(csv.DictReader(open(sys.argv[1])))
tr.sort(key=lambda x: int(x["Start_Timestamp"]))
# first factorization only: up to the first k_perm_in (a solve) or the end
g_tr = [x for x in tr if "k_gemm" in x["Kernel_Name"] or x["Kernel_Name"].startswith("Cijk")]
sched = [r for r in csv.DictReader(open(sys.argv[2])) if r["name"] in ("gemm", "gemm22", "gemmu", "gemmo", "trsm")
         and int(r["tile"]) in (64, 65, 128, 129, 130, 200)]
n = min(len(g_tr), len(sched))
print(f"trace gemm dispatches {len(g_tr)}, schedule gemm launches {len(sched)}; joining {n}")
rows = []
for x, s in zip(g_tr[:n], sched[:n]):
    us = (int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e3
    rows.append(dict(kind=s["name"], tile=int(s["tile"]), nwg=int(s["nwg"]), flops=float(s["flops"]),
                     k=int(s["kmax"]), mn=float(s["mn"]), us=us, kname=x["Kernel_Name"].split("(")[0]))
tot_us = sum(r["us"] for r in rows)
print(f"total {tot_us / 1e3:.1f} ms")


def agg(key, title):
    d = defaultdict(lambda: [0, 0.0, 0.0])
    for r in rows:
        k = key(r)
        d[k][0] += 1
        d[k][1] += r["flops"]
        d[k][2] += r["us"]
    print(f"\n{title}")
    print(f"{'bucket':>26s} {'launches':>8s} {'GFLOP':>9s} {'ms':>8s} {'TF/s':>6s}")
    for k in sorted(d):
        c, f, u = d[k]
        tf = f / (u * 1e-6) / 1e12 if u > 0 and f > 0 else 0
        print(f"{str(k):>26s} {c:8d} {f / 1e9:9.1f} {u / 1e3:8.2f} {tf:6.1f}")


agg(lambda r: (r["kind"], r["tile"]), "by kind, tile")


def nb(r):
    w = r["nwg"]
    for lim in (64, 128, 256, 512, 1024, 2048, 4096, 8192):
        if w <= lim:
            return f"nwg<={lim}"
    return "nwg>8192"


agg(lambda r: (r["tile"], nb(r)), "by tile, tiles per launch")


def kb(r):
    k = r["k"]
    for lim in (32, 64, 128, 256, 384, 512, 1024, 2048, 4096):
        if k <= lim:
            return f"k<={lim}"
    return "k>4096"


agg(lambda r: (r["kind"], kb(r)), "by kind, k")
# wave quantisation estimate for the 128 tiles: fraction of the last wave filled
q = [r for r in rows if r["tile"] in (129, 200) and r["flops"] > 0]
if q:
    eff = sum(r["flops"] for r in q) / sum(r["us"] for r in q) / 1e6
    waste = 0.0
    for r in q:
        waves = r["nwg"] / 512
        full = int(waves)
        frac = waves - full
        if frac > 0:
            waste += r["us"] * (1 - frac) / (full + 1)
    print(f"\nmfma128: {eff:.1f} TF/s over {len(q)} launches; last-wave idle estimate {waste / 1e3:.1f} ms")
