#!/bin/bash
# Round-6 A/B 12 (via gpurun from the repo root): barrier-free panel hand-off with the owner at
# s_setprio 3 (var/pfl2.so), and also with the followers polling at s_sleep 4 (var/pfl3.so, panel
# trace of this one) vs the committed build (var/base4.so).
set -o pipefail
mkdir -p gpurun_out
for v in base4 pfl2 pfl3; do
  SMLU_LIB=$PWD/var/$v.so timeout -k 10 300 python tools/factor_hash.py > gpurun_out/r6_hash_$v.txt 2>gpurun_out/r6_hash_$v.log || { echo hash $v FAIL; tail -5 gpurun_out/r6_hash_$v.log; exit 1; }
  echo "== $v"; cat gpurun_out/r6_hash_$v.txt
done
SMLU_LIB=$PWD/sharedmemsparselu.jl_amd/build_trace/libsmlu_ptrace.so timeout -k 10 300 python tools/panel_trace.py > gpurun_out/panel_trace3.txt 2>gpurun_out/panel_trace3.log || exit 1
tail -5 gpurun_out/panel_trace3.txt
for v in base4 pfl2 pfl3; do
  SMLU_LIB=$PWD/var/$v.so timeout -k 10 120 python tools/c2_bench.py > gpurun_out/r6_c2_$v.json 2>/dev/null || { echo C2 $v FAIL; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r6_c2_$v.json')); print('c2 $v', round(d['refactor_ms_median'],3), round(d['solve_ms_median'],3))"
done
bash tools/ab_libs.sh "var/base4.so var/pfl2.so var/pfl3.so var/base4.so" || exit 1
SMLU_LIB=$PWD/var/pfl3.so timeout -k 10 500 python -u -m pytest tests/test_gpu_kernel_parity.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r6_pfl3_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r6_pfl3_tests.log
exit $rc
