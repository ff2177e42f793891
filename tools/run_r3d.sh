# round-3: GEMM v2 (LDS stride 17 + XCD remap) vs v1, sweep tests, solve timing, refactor bench with/without rocBLAS
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_solve_sweep.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r3d_tests.log 2>&1 || { echo TESTS FAIL; tail -40 gpurun_out/r3d_tests.log; exit 1; }
tail -3 gpurun_out/r3d_tests.log
timeout -k 10 200 python -u tools/solve_timing.py --side 128 > gpurun_out/r3d_solve.log 2>&1 || { echo SOLVE FAIL; tail -20 gpurun_out/r3d_solve.log; exit 1; }
tail -2 gpurun_out/r3d_solve.log
timeout -k 10 300 python bench.py --no-cpu --no-configs > gpurun_out/r3d_bench_default.json 2> gpurun_out/r3d_bench_default.log || { echo BENCH FAIL; tail -20 gpurun_out/r3d_bench_default.log; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r3d_bench_default.json')); print('default', d['ms_per_step'], d['roofline']['frac'], d['kernel_ms_per_step'], d['solve_ms'])"
SMLU_NO_ROCBLAS=1 timeout -k 10 300 python bench.py --no-cpu --no-configs > gpurun_out/r3d_bench_norb.json 2> gpurun_out/r3d_bench_norb.log || { echo BENCH2 FAIL; tail -20 gpurun_out/r3d_bench_norb.log; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r3d_bench_norb.json')); print('norocblas', d['ms_per_step'], d['roofline']['frac'], d['kernel_ms_per_step'], d['solve_ms'])"
