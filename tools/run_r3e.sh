# F22-like GEMM shapes (the refactor's large-K updates) with the refactor's leading dimensions, v1 vs v2;
# then the sweep tests, solve timing and the refactor bench without rocBLAS
set -o pipefail
cd $GRAFT_REPO_ROOT/sharedmemsparselu.jl_amd
S="16384,16384,8192,24576,8192,16384 8192,8192,4096,12288,4096,8192 4096,4096,4096,8192,4096,4096 8192,8192,8192 16000,16000,384"
GB_TILES=129,130 timeout -k 10 200 ./tools/gemm_bench $S > ../gpurun_out/r3e_gemm.txt 2>&1 || { cat ../gpurun_out/r3e_gemm.txt; exit 1; }
cat ../gpurun_out/r3e_gemm.txt
cd ..
timeout -k 10 300 python -u -m pytest tests/test_gpu_solve_sweep.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r3e_tests.log 2>&1 || { echo TESTS FAIL; tail -40 gpurun_out/r3e_tests.log; exit 1; }
tail -2 gpurun_out/r3e_tests.log
timeout -k 10 200 python -u tools/solve_timing.py --side 128 > gpurun_out/r3e_solve.log 2>&1 || { echo SOLVE FAIL; tail -20 gpurun_out/r3e_solve.log; exit 1; }
tail -1 gpurun_out/r3e_solve.log
SMLU_NO_ROCBLAS=1 timeout -k 10 300 python bench.py --no-cpu --no-configs > gpurun_out/r3e_bench_norb.json 2> gpurun_out/r3e_bench_norb.log || { echo BENCH2 FAIL; tail -20 gpurun_out/r3e_bench_norb.log; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r3e_bench_norb.json')); print('norocblas', d['ms_per_step'], d['roofline']['frac'], d['kernel_ms_per_step'], d['solve_ms'], d['solve_8rhs_ms'])"
