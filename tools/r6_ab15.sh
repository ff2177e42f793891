#!/bin/bash
# Round-6 A/B 15 (via gpurun from the repo root): k_bwd_u12 with two rows per lane (var/u12x2.so)
# vs the committed build (var/base5.so): factor and solve hashes (bitwise check), the 128^3 bench
# (1- and 8-rhs solve times), the solve and parity tests.
set -o pipefail
mkdir -p gpurun_out
for v in base5 u12x2; do
  SMLU_LIB=$PWD/var/$v.so timeout -k 10 300 python tools/factor_hash.py > gpurun_out/r6_hash_$v.txt 2>gpurun_out/r6_hash_$v.log || { echo hash $v FAIL; tail -5 gpurun_out/r6_hash_$v.log; exit 1; }
  echo "== $v"; cat gpurun_out/r6_hash_$v.txt
done
for v in base5 u12x2 base5 u12x2; do
  SMLU_LIB=$PWD/var/$v.so timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu --no-configs > gpurun_out/r6_u12_$v.json 2>/dev/null || { echo bench $v FAIL; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r6_u12_$v.json')); print('$v', round(d['ms_per_step'],2), 'solve', round(d['solve_ms'],3), 'solve8', round(d['solve_8rhs_ms'],3))"
done
SMLU_LIB=$PWD/var/u12x2.so timeout -k 10 500 python -u -m pytest tests/test_gpu_solve_sweep.py tests/test_gpu_parity.py tests/test_gpu_reference_suite.py tests/test_gpu_complex.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r6_u12_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r6_u12_tests.log
exit $rc
