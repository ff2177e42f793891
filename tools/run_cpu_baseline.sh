# The default bench line with its CPU baseline, then the direct CPU measurement at the headline size
# (tools/cpu_c3.py) on the GPU box's host cores (via gpurun from the repo root).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/cb_bench.json 2> gpurun_out/cb_bench.log || { tail -5 gpurun_out/cb_bench.log; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/cb_bench.json')); c=d['cpu_baseline']
print('bench', round(d['ms_per_step'],1), 'ms; cpu', c)
"
timeout -k 10 700 python -u tools/cpu_c3.py --cap 200 > gpurun_out/cpu_c3.json 2> gpurun_out/cpu_c3.log || { tail -5 gpurun_out/cpu_c3.log; exit 1; }
cat gpurun_out/cpu_c3.json
