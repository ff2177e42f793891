#!/bin/bash
# Round-6 A/B 16 (via gpurun from the repo root): k_urows on 16-column blocks at three workgroups
# per CU (var/u16.so) vs 32 columns at two (var/base6.so, the committed kernel); the 128^3 bench,
# then the kernel parity tests against u16.
set -o pipefail
mkdir -p gpurun_out
bash tools/ab_libs.sh "var/base6.so var/u16.so var/base6.so var/u16.so" || exit 1
SMLU_LIB=$PWD/var/u16.so timeout -k 10 500 python -u -m pytest tests/test_gpu_kernel_parity.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r6_u16_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r6_u16_tests.log
exit $rc
