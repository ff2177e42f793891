# dev: solve tests (micro fronts) + bench solve times, micro on/off; then the panel PMC passes
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_solve_sweep.py tests/test_gpu_parity.py tests/test_gpu_complex.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3w_tests.log 2>&1 || { echo PYTEST FAIL; tail -40 gpurun_out/r3w_tests.log; exit 1; }
tail -2 gpurun_out/r3w_tests.log
for v in 0 1; do
  if [ $v = 1 ]; then export SMLU_NO_MICRO_SOLVE=1; fi
  timeout -k 10 200 python bench.py --no-cpu --no-configs --steps 2 > gpurun_out/r3w_b$v.json 2> gpurun_out/r3w_b$v.log || { tail -5 gpurun_out/r3w_b$v.log; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r3w_b$v.json')); print('nomicro=$v', round(d['ms_per_step'],1), 'solve', round(d['solve_ms'],2), '8rhs', round(d['solve_8rhs_ms'],2))"
done
unset SMLU_NO_MICRO_SOLVE
bash tools/run_r3v.sh
