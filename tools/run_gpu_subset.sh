# usage: bash tools/run_gpu_subset.sh <log-name> <pytest args...>
set -o pipefail
cd $GRAFT_REPO_ROOT
log=gpurun_out/$1.log; shift
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread "$@" > $log 2>&1
rc=$?
tail -15 $log
exit $rc
