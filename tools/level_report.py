"""Per-level time of one eager factorization (dev): joins a rocprofv3 kernel trace of
tools/pmc_factor.py (SMLU_NO_GRAPH=1, SMLU_DUMP_SCHEDULE=<csv>) with the schedule dump; a level
starts at its k_assemble launch.  Usage: python tools/level_report.py <kernel_trace.csv> <schedule.csv>"""
import csv
import sys
from collections import defaultdict

tr = [x for x in csv.DictReader(open(sys.argv[1])) if x["Kernel_Name"].startswith(("smlu::", "void smlu::", "Cijk"))
      and "k_rowscale" not in x["Kernel_Name"]]
tr.sort(key=lambda x: int(x["Start_Timestamp"]))
sched = list(csv.DictReader(open(sys.argv[2])))
sched = [s for s in sched if s["name"] not in ("sync",)]
n = min(len(tr), len(sched))
lev = -1
per = defaultdict(lambda: defaultdict(float))
span = defaultdict(lambda: [None, None])
cnt = defaultdict(int)
for x, s in zip(tr[:n], sched[:n]):
    if s["name"] == "assemble":
        lev += 1
    us = (int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e3
    per[lev][s["name"]] += us
    cnt[lev] += 1
    a, b = span[lev]
    st, en = int(x["Start_Timestamp"]), int(x["End_Timestamp"])
    span[lev] = [st if a is None else min(a, st), en if b is None else max(b, en)]
print(f"joined {n} of trace {len(tr)} / schedule {len(sched)}")
kinds = sorted({k for d in per.values() for k in d})
print("lvl launches  span_ms " + " ".join(f"{k:>8s}" for k in kinds))
for l in sorted(per):
    sp = (span[l][1] - span[l][0]) / 1e6
    print(f"{l:3d} {cnt[l]:8d} {sp:8.2f} " + " ".join(f"{per[l].get(k, 0) / 1e3:8.2f}" for k in kinds))
