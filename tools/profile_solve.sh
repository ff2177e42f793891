# Kernel trace of the single-vector solve at N^3 (via gpurun from the repo root): rocprofv3 over
# tools/solve_bench.py, then the per-kernel summary of the last solve (tools/ktrace_summary.py).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
N=${1:-128}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/sol_kt -o kt --output-format csv -- python3 tools/solve_bench.py $N > gpurun_out/sol_kt.json 2> gpurun_out/sol_kt.log || { echo SOLVE KT FAIL; tail gpurun_out/sol_kt.log; exit 1; }
f=$(find gpurun_out/sol_kt -name "kt_kernel_trace.csv" | head -1)
python tools/ktrace_summary.py $f > gpurun_out/sol_kt_summary.txt && cat gpurun_out/sol_kt_summary.txt
python tools/solve_levels.py $f > gpurun_out/sol_levels.txt && cat gpurun_out/sol_levels.txt
