set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r02a.log 2>&1
rc=$?
tail -5 gpurun_out/gpu_tests_r02a.log
exit $rc
