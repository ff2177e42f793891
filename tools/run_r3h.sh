# Round-3 full check: every -m gpu test, smoke, then the default bench line (CPU baseline +
# the C1/C2/C5 config lines).  bash tools/run_r3h.sh TAG
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-r3h}
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { echo PYTEST FAIL; tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -3 gpurun_out/${T}_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { echo SMOKE FAIL; tail -20 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
timeout -k 10 420 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.log || { echo BENCH FAIL; tail -20 gpurun_out/${T}_bench.log; exit 1; }
cat gpurun_out/${T}_bench.json
