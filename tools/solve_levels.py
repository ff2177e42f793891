"""Timeline of the last single-vector solve in a rocprofv3 kernel trace (dev): every launch between
the last k_perm_in and the k_perm_out after it, in order, with its duration and the gap before it,
then totals per kernel kind for the forward and backward halves."""
import csv
import sys

r = list(csv.DictReader(open(sys.argv[1])))
r.sort(key=lambda x: int(x["Start_Timestamp"]))
ins = [i for i, x in enumerate(r) if "k_perm_in" in x["Kernel_Name"]]
a = ins[-1]
b = next(i for i in range(a, len(r)) if "k_perm_out" in r[i]["Kernel_Name"])
seg = r[a:b + 1]
t0 = int(seg[0]["Start_Timestamp"])
prev_end = t0
half = "fwd"
tot = {}
gaps = {"fwd": 0.0, "bwd": 0.0}
for x in seg:
    nm = x["Kernel_Name"].split("(")[0].replace("smlu::", "").replace("void ", "")[:30]
    s, e = int(x["Start_Timestamp"]), int(x["End_Timestamp"])
    if "bwd" in nm or "<true" in nm:
        half = "bwd"
    gaps[half] += max(0, s - prev_end) / 1e3
    print(f"{(s - t0) / 1e3:9.1f} us  {(e - s) / 1e3:8.1f} us  gap {(s - prev_end) / 1e3:6.1f}  {nm}")
    tot[(half, nm)] = tot.get((half, nm), 0.0) + (e - s) / 1e3
    prev_end = e
print(f"span {(int(seg[-1]['End_Timestamp']) - t0) / 1e3:.1f} us; gaps fwd {gaps['fwd']:.1f} us, bwd {gaps['bwd']:.1f} us")
for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
    print(f"  {k[0]} {k[1]:32s} {v:9.1f} us")
