# Refactor timing diagnosis, then the default bench line (with its CPU baseline) and the per-launch
# GEMM report (via gpurun from the repo root).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/refactor_timing.py 128 > gpurun_out/rt.txt 2>&1; cat gpurun_out/rt.txt | grep -v amdgpu.ids
timeout -k 10 200 python -u tools/refactor_timing.py 128 profile > gpurun_out/rt_prof.txt 2>&1; cat gpurun_out/rt_prof.txt | grep -v amdgpu.ids
timeout -k 10 300 python bench.py > gpurun_out/r4g_bench.json 2> gpurun_out/r4g_bench.log || { echo BENCH FAIL; tail -20 gpurun_out/r4g_bench.log; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/r4g_bench.json')); c=d['cpu_baseline']
print('bench', round(d['ms_per_step'],1), 'ms; cpu', round(c['headline_seconds'],1), 's', c['sample'])
"
bash tools/profile_gemm_launches.sh > gpurun_out/r4g_gl.txt 2>&1 && tail -20 gpurun_out/r4g_gl.txt
