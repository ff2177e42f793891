# Every -m gpu test without stopping at the first failure (via gpurun from the repo root), one
# process, per-test time limit: bash tools/run_gpu_all.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-all}
timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|SKIPPED" gpurun_out/${T}_tests.log | grep -v PASSED | tail -40
tail -3 gpurun_out/${T}_tests.log
exit $rc
