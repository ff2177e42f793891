#!/bin/bash
# GPU check of the current tree (run through gpurun): the -m gpu suite, smoke(), a short bench.
# Usage: tools/gpu_check.sh TAG [pytest -k expression]
set -o pipefail
TAG=${1:-chk}
K=${2:-}
mkdir -p gpurun_out
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
fi
tail -3 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.log || { tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
python - <<PY
import json; r=json.load(open("gpurun_out/${TAG}_bench.json"))
print("ms_per_step", r["ms_per_step"], "frac", r["roofline"]["frac"], "solve_ms", r["solve_ms"], "solve8", r["solve_8rhs_ms"])
print("kinds", {k: round(v,2) for k,v in r["kernel_ms_per_step"].items()})
PY
