# dev: parity subset + bench A/B for a schedule switch.  bash tools/run_r3l.sh TAG ENVVAR
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-r3l}; V=${2:-SMLU_FUSED_PANEL}
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernel_parity.py tests/test_gpu_parity.py tests/test_gpu_reference_suite.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { echo PYTEST FAIL; tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
for v in ${VALS:-1 0}; do
  env $V=$v timeout -k 10 200 python bench.py --no-cpu --no-configs --steps 3 > gpurun_out/${T}_b$v.json 2> gpurun_out/${T}_b$v.log || { tail -5 gpurun_out/${T}_b$v.log; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/${T}_b$v.json')); print('$V=$v', round(d['ms_per_step'],1), round(d['solve_ms'],2), d.get('launches_per_refactor'), {k: round(v,1) for k,v in d['kernel_ms_per_step'].items()})"
done
