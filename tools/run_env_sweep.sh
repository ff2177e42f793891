# Dev: short 128^3 bench under several environment settings (one line each).
# bash tools/run_env_sweep.sh "VAR=a VAR2=b" "VAR=c" ...
set -o pipefail
cd $GRAFT_REPO_ROOT
i=0
for cfg in "$@"; do
  i=$((i+1))
  env $cfg timeout -k 10 300 python bench.py --no-cpu --steps 3 --warmup 1 > gpurun_out/sweep_$i.json 2> gpurun_out/sweep_$i.log || { echo "FAIL $cfg"; tail -5 gpurun_out/sweep_$i.log; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/sweep_$i.json')); print('$cfg', round(d['ms_per_step'],1), {k: round(v,1) for k,v in d['kernel_ms_per_step'].items()})"
done
