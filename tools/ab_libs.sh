#!/bin/bash
# Dev A/B of library variants (via gpurun from the repo root): the 128^3 bench with each given
# .so (SMLU_LIB), one line per variant with the per-kind kernel times, then optionally a pytest
# selection against the LAST variant.
# Usage: tools/ab_libs.sh "var/base.so var/x.so var/y.so@KNOB=1" [pytest -k expression]
# (an entry lib@NAME=VALUE runs that variant with the environment variable set)
set -o pipefail
mkdir -p gpurun_out
LIBS=$1
K=${2:-}
n=0
for E in $LIBS; do
  n=$((n + 1))
  L=${E%%@*}
  EV=""
  [ "$E" != "$L" ] && EV=${E#*@}
  T=$(basename $L .so)_$n
  env $EV SMLU_LIB=$PWD/$L timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu --no-configs \
    > gpurun_out/ab_$T.json 2> gpurun_out/ab_$T.log || { echo "$T FAILED"; tail -20 gpurun_out/ab_$T.log; exit 1; }
  python - <<PY
import json; r=json.load(open("gpurun_out/ab_$T.json"))
print("$T", "ms", round(r["ms_per_step"], 2), "frac", round(r["roofline"]["frac"], 4), "solve", r.get("solve_ms"))
print("   ", {k: round(v, 2) for k, v in r["kernel_ms_per_step"].items()})
PY
done
if [ -n "$K" ]; then
  SMLU_LIB=$PWD/$L timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" \
    > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
  tail -3 gpurun_out/ab_tests.log
fi
