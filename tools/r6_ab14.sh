#!/bin/bash
# Round-6 A/B 14 (via gpurun from the repo root): the sentinel hand-off of A/B 13 (var/pfl4.so) and
# the same with only the next owner following column by column, the later waves waiting for the
# whole block (var/pfl5.so, panel trace of this one) vs the committed build (var/base4.so).
set -o pipefail
mkdir -p gpurun_out
for v in base4 pfl5; do
  SMLU_LIB=$PWD/var/$v.so timeout -k 10 300 python tools/factor_hash.py > gpurun_out/r6_hash_$v.txt 2>gpurun_out/r6_hash_$v.log || { echo hash $v FAIL; tail -5 gpurun_out/r6_hash_$v.log; exit 1; }
  echo "== $v"; cat gpurun_out/r6_hash_$v.txt
done
SMLU_LIB=$PWD/sharedmemsparselu.jl_amd/build_trace/libsmlu_ptrace.so timeout -k 10 300 python tools/panel_trace.py > gpurun_out/panel_trace3.txt 2>gpurun_out/panel_trace3.log || exit 1
tail -5 gpurun_out/panel_trace3.txt
for v in base4 pfl5; do
  SMLU_LIB=$PWD/var/$v.so timeout -k 10 120 python tools/c2_bench.py > gpurun_out/r6_c2_$v.json 2>/dev/null || { echo C2 $v FAIL; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r6_c2_$v.json')); print('c2 $v', round(d['refactor_ms_median'],3), round(d['solve_ms_median'],3))"
done
bash tools/ab_libs.sh "var/base4.so var/pfl4.so var/pfl5.so var/base4.so var/pfl4.so var/pfl5.so" || exit 1
SMLU_LIB=$PWD/var/pfl5.so timeout -k 10 500 python -u -m pytest tests/test_gpu_kernel_parity.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r6_pfl5_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r6_pfl5_tests.log
exit $rc
