#!/bin/bash
# Round-6 A/B 5 (via gpurun from the repo root): k_urows with 16-column blocks for launches of at
# most SMLU_UROWS_NARROW 32-column blocks (0 = never, 512, 4096 = nearly always) -- C2, the 128^3
# bench, then the kernel parity tests against the always-narrow variant.
set -o pipefail
mkdir -p gpurun_out
for v in base2 nar0 nar512 nar4096; do
  SMLU_LIB=$PWD/var/$v.so timeout -k 10 120 python tools/c2_bench.py > gpurun_out/r6_c2_$v.json 2>/dev/null || { echo C2 $v FAIL; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r6_c2_$v.json')); print('c2 $v', round(d['refactor_ms_median'],3), round(d['solve_ms_median'],3))"
done
bash tools/ab_libs.sh "var/base2.so var/nar0.so var/nar512.so var/nar4096.so" || exit 1
SMLU_LIB=$PWD/var/nar4096.so timeout -k 10 500 python -u -m pytest tests/test_gpu_kernel_parity.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r6_nar_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r6_nar_tests.log
exit $rc
