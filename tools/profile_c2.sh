# Kernel trace of C2 (2D Poisson 512^2) refactor + solve (via gpurun from the repo root).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/c2_kt -o kt --output-format csv -- python3 tools/c2_bench.py > gpurun_out/c2_kt.json 2> gpurun_out/c2_kt.log || { echo C2 KT FAIL; tail gpurun_out/c2_kt.log; exit 1; }
cat gpurun_out/c2_kt.json | cut -c1-400
f=$(find gpurun_out/c2_kt -name "kt_kernel_trace.csv" | head -1)
python tools/ktrace_summary.py $f > gpurun_out/c2_kt_summary.txt && cat gpurun_out/c2_kt_summary.txt
