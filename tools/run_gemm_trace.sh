# Kernel trace of one eager 128^3 factorization + the schedule dump (dev):
# bash tools/run_gemm_trace.sh TAG ; then python tools/gemm_dispatch_report.py gpurun_out/TAG/kt_kernel_trace.csv gpurun_out/TAG_sched.csv
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-gt}
export SMLU_NO_GRAPH=1 SMLU_DUMP_SCHEDULE=$GRAFT_REPO_ROOT/gpurun_out/${T}_sched.csv
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/$T -o kt --output-format csv -- python3 tools/pmc_factor.py 128 > gpurun_out/$T.log 2>&1
