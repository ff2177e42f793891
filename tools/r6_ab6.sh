#!/bin/bash
# Round-6 A/B 6 (via gpurun from the repo root): k_urows with the first R block's L fragments
# issued before the T step (urp: 2 workgroups per CU; urp1: 1 per CU, NL_{u+1} prefetched during
# R) vs the committed kernel -- the 128^3 bench, then the kernel parity tests against urp.
set -o pipefail
mkdir -p gpurun_out
bash tools/ab_libs.sh "var/base2.so var/urp1.so var/urp.so var/base2.so" || exit 1
SMLU_LIB=$PWD/var/urp.so timeout -k 10 500 python -u -m pytest tests/test_gpu_kernel_parity.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r6_urp_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r6_urp_tests.log
exit $rc
