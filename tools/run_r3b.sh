# round-3 check: GEMM tile v2 vs v1 (+PMC), the solve sweep tests, 128^3 solve timing
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/run_gemm_v2.sh > gpurun_out/r3b_gemm.log 2>&1 || { echo GEMM FAIL; tail -20 gpurun_out/r3b_gemm.log; exit 1; }
tail -14 gpurun_out/r3b_gemm.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_solve_sweep.py tests/test_gpu_kernel_parity.py -x -v --timeout 120 --timeout-method thread -k "sweep or sequence or redecides" > gpurun_out/r3b_tests.log 2>&1 || { echo TESTS FAIL; tail -40 gpurun_out/r3b_tests.log; exit 1; }
tail -3 gpurun_out/r3b_tests.log
timeout -k 10 200 python -u tools/solve_timing.py --side 128 > gpurun_out/r3b_solve.log 2>&1 || { echo SOLVE FAIL; tail -20 gpurun_out/r3b_solve.log; exit 1; }
tail -2 gpurun_out/r3b_solve.log
