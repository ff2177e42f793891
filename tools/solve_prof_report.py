"""Per-solve kernel breakdown from a rocprofv3 kernel-trace database of tools/solve_timing.py:
each solve is the dispatch run from k_perm_in to k_perm_out; prints the first solve of every
batch width (grid_y of k_perm_in)."""
import collections
import sqlite3
import sys

db = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof_solve/run_results.db"
c = sqlite3.connect(db)
rows = list(c.execute("select name, start, end, grid_y from kernels order by start"))
seen, cur = set(), None
for name, s, e, gy in rows:
    if "k_perm_in" in name:
        cur = {"nr": gy, "t0": s, "k": collections.Counter(), "c": collections.Counter()}
    if cur is None:
        continue
    key = name.split("(")[0].replace("smlu::", "").replace("void ", "")
    cur["k"][key] += (e - s) / 1e6
    cur["c"][key] += 1
    if "k_perm_out" in name:
        if cur["nr"] not in seen:
            seen.add(cur["nr"])
            print(f"nrhs {cur['nr']}: wall {(e - cur['t0']) / 1e6:.2f} ms, kernels {sum(cur['k'].values()):.2f} ms")
            for k, v in cur["k"].most_common(8):
                print(f"    {k:32s} {cur['c'][k]:5d} {v:8.2f} ms")
        cur = None
