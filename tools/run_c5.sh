# BASELINE C5 at its stated size (via gpurun from the repo root): 1000 refactors of 128^3.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 1000 python -u tools/c5_steady.py --n 128 --reps 1000 > gpurun_out/c5_128_1000.json 2> gpurun_out/c5_128_1000.log || { echo C5 FAIL; tail -20 gpurun_out/c5_128_1000.log; exit 1; }
tail -3 gpurun_out/c5_128_1000.log
python -c "
import json; d=json.load(open('gpurun_out/c5_128_1000.json')); print(json.dumps({k: d[k] for k in ('refactor_ms','device_mem_GB','residual_after_last','steady_state_nnzLU_per_s')}))
"
