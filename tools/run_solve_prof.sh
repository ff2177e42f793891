# Kernel trace of tools/solve_timing.py (one MI355X, via gpurun from the repo root); the CSV is
# summarised per solve by tools/solve_trace_report.py on the host.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-sp}
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${T}_kt -o kt --output-format csv -- python3 tools/solve_timing.py --reps 2 > gpurun_out/${T}_kt.log 2>&1 || { tail -20 gpurun_out/${T}_kt.log; exit 1; }
tail -1 gpurun_out/${T}_kt.log
