# Solve timings for the sweep / per-block batch variants (via gpurun from the repo root).
set -o pipefail
cd $GRAFT_REPO_ROOT
N=${1:-128}
timeout -k 10 200 python tools/solve_bench.py $N > gpurun_out/solve_v1.json 2> gpurun_out/solve_v1.log || exit 1
cat gpurun_out/solve_v1.json
SMLU_SWEEP_MAX_RHS=8 timeout -k 10 200 python tools/solve_bench.py $N > gpurun_out/solve_v8.json 2> gpurun_out/solve_v8.log || exit 1
cat gpurun_out/solve_v8.json
SMLU_DIAG_INV=1 timeout -k 10 200 python tools/solve_bench.py $N > gpurun_out/solve_inv.json 2> gpurun_out/solve_inv.log || exit 1
cat gpurun_out/solve_inv.json
