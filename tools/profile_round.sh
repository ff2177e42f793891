# Round profile on one MI355X (via gpurun from the repo root): GPU tests, full bench (with the
# CPU baseline), rocprofv3 kernel stats of the bench, and the two PMC passes (FETCH_SIZE,
# WRITE_SIZE) restricted to the k_gemm* dispatches of one eager factorization.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
N=${1:-128}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tgpu.log 2>&1 || { echo PYTEST FAIL; tail -30 gpurun_out/tgpu.log; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/p_bench.json 2> gpurun_out/p_bench.log || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p_kt -o kt --output-format csv -- python3 bench.py --no-cpu --steps 2 --warmup 1 > gpurun_out/p_kt.json 2> gpurun_out/p_kt.log || exit 1
export SMLU_NO_GRAPH=1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-include-regex "k_gemm|Cijk" -d gpurun_out/pmc_${c}_$N -o pmc \
    --output-format csv -- python3 tools/pmc_factor.py $N > gpurun_out/pmc_${c}_$N.log 2>&1 || exit 1
done
# the same two counters over every kernel of the factorization: whole-refactor HBM bytes
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c -d gpurun_out/pmcall_${c}_$N -o pmc \
    --output-format csv -- python3 tools/pmc_factor.py $N > gpurun_out/pmcall_${c}_$N.log 2>&1 || exit 1
done
