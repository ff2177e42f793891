# Solve change check on one MI355X (via gpurun from the repo root): sweep + parity GPU tests, then a
# kernel trace of tools/solve_timing.py (summarised on the host by tools/solve_trace_report.py).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-sc}
timeout -k 10 400 python -u -m pytest tests/test_gpu_solve_sweep.py tests/test_gpu_parity.py tests/test_gpu_reference_suite.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_t.log 2>&1 || { echo PYTEST FAIL; tail -30 gpurun_out/${T}_t.log; exit 1; }
tail -2 gpurun_out/${T}_t.log
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${T}_kt -o kt --output-format csv -- python3 tools/solve_timing.py --reps 2 > gpurun_out/${T}_kt.log 2>&1 || { tail -20 gpurun_out/${T}_kt.log; exit 1; }
grep side gpurun_out/${T}_kt.log
