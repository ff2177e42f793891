#!/bin/bash
# Round-6 A/B 2 (via gpurun from the repo root): level overlap (small fronts next to the blocked
# fronts' chain, factor and solve) -- var/base.so vs var/ovl2.so: C2, the 128^3 solve and refactor;
# then every -m gpu test against the default library.
set -o pipefail
mkdir -p gpurun_out
for v in base ovl2; do
  SMLU_LIB=$PWD/var/$v.so timeout -k 10 120 python tools/c2_bench.py > gpurun_out/r6_c2_$v.json 2>/dev/null || { echo C2 $v FAIL; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r6_c2_$v.json')); print('c2 $v', round(d['refactor_ms_median'],3), round(d['solve_ms_median'],3))"
  SMLU_LIB=$PWD/var/$v.so timeout -k 10 200 python -u tools/solve_bench.py 128 > gpurun_out/r6_solve3_$v.json 2> gpurun_out/r6_solve3_$v.log || { echo SOLVE $v FAIL; tail gpurun_out/r6_solve3_$v.log; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r6_solve3_$v.json')); print('solve128 $v', round(d['solve_ms'],3), round(d['solve8_ms'],3))"
done
bash tools/ab_libs.sh "var/base.so var/ovl2.so" || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6h_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r6h_tests.log
exit $rc
