"""Per-launch GEMM efficiency of one refactor (dev): pairs the schedule dump (SMLU_DUMP_LAUNCHES=
<csv>, written when the schedule is built) with a rocprofv3 kernel trace of the same run, in
dispatch order, and reports TFLOP/s per launch kind and per launch size class.

    python tools/gemm_launch_report.py launches.csv kt_kernel_trace.csv
"""
import csv
import sys
from collections import defaultdict

KIND = {8: "gemm(in-block)", 18: "gemmu", 19: "gemmo(trailing)", 15: "gemm22(F22)", 7: "trsm(gemm-form)"}
dump = list(csv.DictReader(open(sys.argv[1])))
tr = list(csv.DictReader(open(sys.argv[2])))
tr.sort(key=lambda x: int(x["Start_Timestamp"]))
starts = [i for i, x in enumerate(tr) if "k_rowscale" in x["Kernel_Name"]]
a = starts[-1]
b = next((i for i in range(a, len(tr)) if "k_perm_in" in tr[i]["Kernel_Name"]), len(tr))
disp = [x for x in tr[a:b] if "k_gemm" in x["Kernel_Name"]]
gl = [d for d in dump if int(d["tile"]) >= 0]
print(f"GEMM launches in the schedule {len(gl)}, GEMM dispatches in the last refactor {len(disp)}")
n = min(len(gl), len(disp))
agg = defaultdict(lambda: [0.0, 0.0, 0])
size = defaultdict(lambda: [0.0, 0.0, 0])
for d, x in zip(gl[:n], disp[:n]):
    us = (int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e3
    fl = float(d["flops"])
    if fl <= 0:
        continue
    k = KIND.get(int(d["kind"]), d["kind"])
    agg[k][0] += fl
    agg[k][1] += us
    agg[k][2] += 1
    t = int(d["nwg"])
    cls = "<256 tiles" if t < 256 else "<1024" if t < 1024 else "<8192" if t < 8192 else ">=8192"
    size[(k, cls)][0] += fl
    size[(k, cls)][1] += us
    size[(k, cls)][2] += 1
for k, (fl, us, c) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"{k:18s} {c:5d} launches {us / 1e3:8.2f} ms {fl / 1e12:7.3f} TFLOP {fl / us / 1e6:6.1f} TFLOP/s")
for (k, cls), (fl, us, c) in sorted(size.items()):
    print(f"  {k:18s} {cls:11s} {c:5d} launches {us / 1e3:8.2f} ms {fl / us / 1e6:6.1f} TFLOP/s")
