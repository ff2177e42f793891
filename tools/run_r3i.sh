# per-dispatch GEMM report of one eager 128^3 factorization with the hand-written tiles only
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/run_gemm_trace.sh r3i || { tail -20 gpurun_out/r3i.log; exit 1; }
f=$(ls gpurun_out/r3i/*kernel_trace.csv 2>/dev/null | head -1)
[ -z "$f" ] && f=$(find gpurun_out/r3i -name '*kernel_trace.csv' | head -1)
python3 tools/gemm_dispatch_report.py $f gpurun_out/r3i_sched.csv > gpurun_out/r3i_report.txt 2>&1
head -40 gpurun_out/r3i_report.txt
