# Solve-path sweep on one MI355X (via gpurun from the repo root): solve-path GPU tests, then
# tools/solve_timing.py once per environment setting given ("-" = defaults).
#   bash tools/run_solve_sweep.sh TAG - SMLU_SOLVE_STEPS=1 SMLU_SOLVE_BIGWORK=32768 ...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=$1; shift
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_reference_suite.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_t.log 2>&1 || { echo PYTEST FAIL; tail -30 gpurun_out/${T}_t.log; exit 1; }
tail -1 gpurun_out/${T}_t.log
k=0
for e in "$@"; do
  k=$((k+1))
  if [ "$e" = "-" ]; then set -- ; else export "$e"; fi
  timeout -k 10 200 python tools/solve_timing.py --reps 3 > gpurun_out/${T}_solve_$k.txt 2>&1 || { tail -20 gpurun_out/${T}_solve_$k.txt; exit 1; }
  echo "$e $(tail -1 gpurun_out/${T}_solve_$k.txt)"
  [ "$e" = "-" ] || unset "${e%%=*}"
done
