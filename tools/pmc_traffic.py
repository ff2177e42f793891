#!/usr/bin/env python3
"""Summarise the PMC passes of tools/profile_pmc.sh into profiles/<round>/pmc_gemm_<N>.json.

HBM bytes per the MI355X guide's HBM/rocprofv3 section: FETCH_SIZE and WRITE_SIZE are in KiB,
collected in separate passes; on gfx950 FETCH_SIZE counts 1/2 of the bytes of wide reads, so
it is doubled; WRITE_SIZE is taken as is.  Usage: pmc_traffic.py N ROUND_DIR
"""
import csv
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import kernel_source_sha  # noqa: E402

N = int(sys.argv[1])
out_dir = sys.argv[2]
base = "gpurun_out"


def short(name):
    """rocBLAS/Tensile kernel names are several hundred characters: keep the macro tile and WGM."""
    if name.startswith("Cijk_"):
        mt = re.search(r"_MT(\w+?)_", name)
        wg = re.search(r"_WGM(\d+)", name)
        return f"rocblas dgemm MT{mt.group(1) if mt else '?'} WGM{wg.group(1) if wg else '?'}"
    return name


def load(counter):
    """Per-kernel totals of the Schur-update GEMMs (the <false> instantiations; the <true> ones
    are the GEMM-form triangular solves, accounted as "trsm")."""
    path = os.path.join(base, f"pmc_{counter}_{N}", "pmc_counter_collection.csv")
    per = {}
    for r in csv.DictReader(open(path)):
        name = short(r["Kernel_Name"].split("(")[0])
        if "<true" in name:   # TRSM forms: first template argument true
            continue
        d = per.setdefault(name, [0, 0.0])
        d[0] += 1
        d[1] += float(r["Counter_Value"])
    return per


def factor_stats():
    txt = open(os.path.join(base, f"pmc_FETCH_SIZE_{N}.log")).read()
    m = re.search(r"gemm_launches=(\d+) gemm_bytes=([\d.e+]+) gemm_flops=([\d.e+]+)", txt)
    return int(m.group(1)), float(m.group(2)), float(m.group(3))


fetch, write = load("FETCH_SIZE"), load("WRITE_SIZE")
launches, alg_bytes, flops = factor_stats()
n = sum(v[0] for v in fetch.values())
fkb = sum(v[1] for v in fetch.values())
wkb = sum(v[1] for v in write.values())
hbm = 2.0 * fkb * 1024 + wkb * 1024
res = {
    "workload": f"3D Poisson {N}^3, one numeric factorization (eager launches)",
    "kernels": {k: {"launches": fetch[k][0], "fetch_kib_raw": fetch[k][1],
                    "write_kib_raw": write.get(k, [0, 0.0])[1]} for k in fetch},
    "launches": n, "launches_expected": launches,
    "fetch_kib_raw": fkb, "write_kib_raw": wkb,
    "hbm_bytes_total": hbm, "hbm_bytes_per_launch": hbm / n,
    "algorithmic_bytes_total": alg_bytes, "algorithmic_bytes_per_launch": alg_bytes / launches,
    "traffic_over_algorithmic": hbm / alg_bytes,
    "gemm_flops": flops,
    "correction": "FETCH_SIZE x2 (gfx950 wide-read tally), KiB -> bytes; WRITE_SIZE as is",
    "kernels_sha": kernel_source_sha(),
}
# whole factorization (every kernel, incl. the memset fills): HBM bytes per refactor
if os.path.exists(os.path.join(base, f"pmcall_FETCH_SIZE_{N}", "pmc_counter_collection.csv")):
    def load_all(counter):
        per = {}
        path = os.path.join(base, f"pmcall_{counter}_{N}", "pmc_counter_collection.csv")
        for r in csv.DictReader(open(path)):
            name = short(r["Kernel_Name"].split("(")[0])
            per[name] = per.get(name, 0.0) + float(r["Counter_Value"])
        return per
    fa, wa = load_all("FETCH_SIZE"), load_all("WRITE_SIZE")
    tot = {k: 2.0 * fa.get(k, 0.0) * 1024 + wa.get(k, 0.0) * 1024 for k in set(fa) | set(wa)}
    res["refactor_all_kernels"] = {
        "hbm_bytes": sum(tot.values()),
        "fetch_bytes": 2.0 * sum(fa.values()) * 1024, "write_bytes": sum(wa.values()) * 1024,
        "by_kernel_top": dict(sorted(tot.items(), key=lambda kv: -kv[1])[:12]),
        "note": "one eager factorization (first factorization incl. k_rowscale), every kernel",
    }
os.makedirs(out_dir, exist_ok=True)
with open(os.path.join(out_dir, f"pmc_gemm_{N}.json"), "w") as fh:
    json.dump(res, fh, indent=1)
print(json.dumps({k: v for k, v in res.items() if k != "kernels"}, indent=1))
