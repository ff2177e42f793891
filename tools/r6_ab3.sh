#!/bin/bash
# Round-6 A/B 3 (via gpurun from the repo root): the small-front threshold kSmallM 128 / 96 / 64
# (fronts up to that order factored whole in LDS by k_front_small) -- C2 and the 128^3 bench.
set -o pipefail
mkdir -p gpurun_out
for v in base2 small96 small64; do
  SMLU_LIB=$PWD/var/$v.so timeout -k 10 120 python tools/c2_bench.py > gpurun_out/r6_c2_$v.json 2>/dev/null || { echo C2 $v FAIL; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r6_c2_$v.json')); print('c2 $v', round(d['refactor_ms_median'],3), round(d['solve_ms_median'],3))"
done
bash tools/ab_libs.sh "var/base2.so var/small96.so var/small64.so" || exit 1
