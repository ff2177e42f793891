# Dev: sweep timing marks + solve timing (via gpurun from the repo root)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-st}
timeout -k 10 200 python tools/sweep_trace.py > gpurun_out/${T}_trace.txt 2>&1 || { tail -20 gpurun_out/${T}_trace.txt; exit 1; }
cat gpurun_out/${T}_trace.txt | grep -v Warning
timeout -k 10 200 python tools/solve_timing.py --reps 3 > gpurun_out/${T}_solve.txt 2>&1 || { tail -5 gpurun_out/${T}_solve.txt; exit 1; }
tail -1 gpurun_out/${T}_solve.txt
