# Solve check on one MI355X (via gpurun from the repo root): solve-path GPU tests, solve timing
# with graphs on and off, then a kernel trace of the solve timing.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-sc}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_reference_suite.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_t.log 2>&1 || { echo PYTEST FAIL; tail -30 gpurun_out/${T}_t.log; exit 1; }
tail -2 gpurun_out/${T}_t.log
timeout -k 10 200 python tools/solve_timing.py > gpurun_out/${T}_solve.txt 2>&1 || { tail -20 gpurun_out/${T}_solve.txt; exit 1; }
tail -1 gpurun_out/${T}_solve.txt
SMLU_NO_GRAPH=1 timeout -k 10 200 python tools/solve_timing.py > gpurun_out/${T}_solve_nograph.txt 2>&1 || exit 1
tail -1 gpurun_out/${T}_solve_nograph.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_kt -o kt --output-format csv -- python3 tools/solve_timing.py --reps 2 > gpurun_out/${T}_kt.log 2>&1 || exit 1
