"""Summarise a rocprofv3 kernel trace of bench.py (dev): per-kernel totals of the last
refactor and of the last solve.  Usage: python tools/ktrace_summary.py gpurun_out/<dir>/kt_kernel_trace.csv"""
import csv
import sys

r = list(csv.DictReader(open(sys.argv[1])))
r.sort(key=lambda x: int(x["Start_Timestamp"]))


def name(x):
    return x["Kernel_Name"].split("(")[0].replace("smlu::", "").replace("void ", "")[:26]


def summary(seg, title):
    tot, cnt = {}, {}
    for x in seg:
        n = name(x)
        tot[n] = tot.get(n, 0) + (int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e6
        cnt[n] = cnt.get(n, 0) + 1
    span = (int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / 1e6
    print(f"{title}: span {span:.1f} ms, busy {sum(tot.values()):.1f} ms, {len(seg)} launches")
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1])[:14]:
        print(f"  {k:28s} {v:8.2f} ms {cnt[k]:6d}  avg {1e3 * v / cnt[k]:8.1f} us")


fac = [i for i, x in enumerate(r) if "k_rowscale" in x["Kernel_Name"]]
sol = [i for i, x in enumerate(r) if "k_perm_in" in x["Kernel_Name"]]
a = fac[-1]
b = min([i for i in sol if i > a], default=len(r))
summary(r[a:b], "refactor")
if sol:
    s0 = sol[-1]
    e = max(i for i, x in enumerate(r) if "k_perm_out" in x["Kernel_Name"])
    summary(r[s0:e + 1], "solve")
