# Dev loop on one MI355X: parity subset + short bench + per-level trace of one eager factorization.
# bash tools/run_dev_round.sh TAG [pytest files...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-d}; shift
bash tools/run_quick.sh $T "$@" || exit 1
bash tools/run_gemm_trace.sh ${T}_gt || exit 1
python tools/level_report.py gpurun_out/${T}_gt/kt_kernel_trace.csv gpurun_out/${T}_gt_sched.csv > gpurun_out/${T}_levels.txt
python tools/gemm_dispatch_report.py gpurun_out/${T}_gt/kt_kernel_trace.csv gpurun_out/${T}_gt_sched.csv > gpurun_out/${T}_gemm.txt
