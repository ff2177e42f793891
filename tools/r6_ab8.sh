#!/bin/bash
# Round-6 A/B 8 (via gpurun from the repo root): fused panel whose applying waves read the block's
# pivots and multipliers in one LDS round trip (var/plds.so) vs the committed build; C2, the 128^3
# bench, then the kernel parity tests against plds.
set -o pipefail
mkdir -p gpurun_out
for v in base3 plds; do
  SMLU_LIB=$PWD/var/$v.so timeout -k 10 120 python tools/c2_bench.py > gpurun_out/r6_c2_$v.json 2>/dev/null || { echo C2 $v FAIL; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r6_c2_$v.json')); print('c2 $v', round(d['refactor_ms_median'],3), round(d['solve_ms_median'],3))"
done
bash tools/ab_libs.sh "var/base3.so var/plds.so var/base3.so var/plds.so" || exit 1
SMLU_LIB=$PWD/var/plds.so timeout -k 10 500 python -u -m pytest tests/test_gpu_kernel_parity.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r6_plds_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r6_plds_tests.log
exit $rc
