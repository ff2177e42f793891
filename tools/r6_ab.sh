#!/bin/bash
# Round-6 A/B (via gpurun from the repo root): GEMM tiles in isolation (zero-init 137/139 vs
# 131/135), the 128^3 bench with the base / zero-init-trailing libraries, the solve with the
# base / 8-wave sweep libraries, and the sweep parity tests against the 8-wave library.
set -o pipefail
mkdir -p gpurun_out
bash tools/gemm_ab.sh r6zi 131,137,135,139 > /dev/null 2>&1 || { echo GEMM AB FAIL; exit 1; }
bash tools/ab_libs.sh "var/base.so var/zi.so" || exit 1
for v in base wk8; do
  SMLU_LIB=$PWD/var/$v.so timeout -k 10 200 python -u tools/solve_bench.py 128 > gpurun_out/r6_solve_$v.json 2> gpurun_out/r6_solve_$v.log || { echo SOLVE $v FAIL; tail gpurun_out/r6_solve_$v.log; exit 1; }
  echo "$v $(cat gpurun_out/r6_solve_$v.json | cut -c1-300)"
done
SMLU_LIB=$PWD/var/wk8.so timeout -k 10 400 python -u -m pytest tests/test_gpu_solve_sweep.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r6_wk8_tests.log 2>&1 || { tail -30 gpurun_out/r6_wk8_tests.log; exit 1; }
tail -2 gpurun_out/r6_wk8_tests.log
