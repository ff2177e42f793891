# dev: parity subset with SMLU_FUSED_PANEL=2 + bench A/B 2 vs 1
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export SMLU_FUSED_PANEL=2
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernel_parity.py tests/test_gpu_parity.py tests/test_gpu_reference_suite.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3t_tests.log 2>&1 || { echo PYTEST FAIL; tail -40 gpurun_out/r3t_tests.log; exit 1; }
tail -2 gpurun_out/r3t_tests.log
for v in 2 1; do
  SMLU_FUSED_PANEL=$v timeout -k 10 200 python bench.py --no-cpu --no-configs --steps 3 > gpurun_out/r3t_b$v.json 2> gpurun_out/r3t_b$v.log || { tail -5 gpurun_out/r3t_b$v.log; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r3t_b$v.json')); print('P=$v', round(d['ms_per_step'],1), round(d['solve_ms'],2), d.get('launches_per_refactor'), {k: round(v,1) for k,v in d['kernel_ms_per_step'].items()})"
done
