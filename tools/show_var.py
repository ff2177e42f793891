"""Dev: one line per bench variant JSON under gpurun_out/."""
import glob, json, sys
for f in sorted(glob.glob("gpurun_out/var_*.json")):
    d = json.load(open(f))
    k = d["kernel_ms_per_step"]
    print(f, round(d["ms_per_step"], 1), round(d["roofline"]["achieved"], 2), round(d["solve_ms"], 1),
          {a: round(b, 1) for a, b in k.items()})
