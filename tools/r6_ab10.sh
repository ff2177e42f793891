#!/bin/bash
# Round-6 A/B 10 (via gpurun from the repo root): the 128 tile with its B-fragment reads kept as
# separate ds_read_b64 (var/b64.so) vs the committed build (var/base4.so): LDS-conflict PMC pass of
# the new build, C2, the 128^3 bench, kernel parity tests.
set -o pipefail
mkdir -p gpurun_out
rm -rf gpurun_out/pmcsq_128
bash tools/pmc_sq.sh || exit 1
for v in base4 b64; do
  SMLU_LIB=$PWD/var/$v.so timeout -k 10 120 python tools/c2_bench.py > gpurun_out/r6_c2_$v.json 2>/dev/null || { echo C2 $v FAIL; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r6_c2_$v.json')); print('c2 $v', round(d['refactor_ms_median'],3), round(d['solve_ms_median'],3))"
done
bash tools/ab_libs.sh "var/base4.so var/b64.so var/base4.so var/b64.so" || exit 1
SMLU_LIB=$PWD/var/b64.so timeout -k 10 500 python -u -m pytest tests/test_gpu_kernel_parity.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r6_b64_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r6_b64_tests.log
exit $rc
