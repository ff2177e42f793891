# dev: timing of the panel / in-block overlap experiment (SMLU_DEV_PGOVL=1 is numerically wrong)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in 0 1; do
  if [ $v = 1 ]; then export SMLU_DEV_PGOVL=1; fi
  timeout -k 10 200 python bench.py --no-cpu --no-configs --steps 3 > gpurun_out/r3y_b$v.json 2> gpurun_out/r3y_b$v.log || { tail -5 gpurun_out/r3y_b$v.log; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r3y_b$v.json')); print('ovl=$v', round(d['ms_per_step'],1), d.get('launches_per_refactor'), {k: round(v,1) for k,v in d['kernel_ms_per_step'].items()})"
done
