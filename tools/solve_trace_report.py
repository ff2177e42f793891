"""Per-solve kernel breakdown from a rocprofv3 kernel-trace CSV of tools/solve_timing.py: each
solve is the dispatch run from k_perm_in to k_perm_out; prints the first timed single-vector
solve (second k_perm_in with grid_y 1): per kernel name count / busy ms, and the idle gaps.

    python tools/solve_trace_report.py gpurun_out/sp_kt/.../kt_kernel_trace.csv [--seq]
"""
import collections
import csv
import sys

path = sys.argv[1]
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
solves, cur = [], None
for r in rows:
    name = r["Kernel_Name"]
    if "k_perm_in" in name:
        cur = []
    if cur is None:
        continue
    cur.append((name.split("(")[0].replace("smlu::", "").replace("void ", ""), int(r["Start_Timestamp"]),
                int(r["End_Timestamp"]), int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0)))
    if "k_perm_out" in name:
        solves.append(cur)
        cur = None
single = [s for s in solves][:3]
s = single[1] if len(single) > 1 else single[0]
t0, t1 = s[0][1], s[-1][2]
busy = collections.Counter()
cnt = collections.Counter()
gap = 0
prev = t0
for k, a, b, g in s:
    busy[k] += (b - a) / 1e6
    cnt[k] += 1
    gap += max(0, a - prev) / 1e6
    prev = max(prev, b)
print(f"wall {(t1 - t0) / 1e6:.3f} ms, kernels {sum(busy.values()):.3f} ms, gaps {gap:.3f} ms, launches {len(s)}")
for k, v in busy.most_common():
    print(f"  {k:40s} {cnt[k]:5d} {v:8.3f} ms")
if "--seq" in sys.argv:
    for k, a, b, g in s:
        print(f"  {(a - t0) / 1e3:9.1f} us {(b - a) / 1e3:8.1f} us  grid {g:8d}  {k}")
