# Dev loop on one MI355X: parity subset + a short 128^3 bench (no CPU baseline).
# bash tools/run_quick.sh TAG [pytest files...]
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-q}; shift
files=${@:-tests/test_gpu_parity.py tests/test_gpu_kernel_parity.py tests/test_gpu_reference_suite.py}
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread $files > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
timeout -k 10 300 python bench.py --no-cpu --steps 3 --warmup 1 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.log || { tail -20 gpurun_out/${T}_bench.log; exit 1; }
python - <<PY
import json; d=json.load(open("gpurun_out/${T}_bench.json"))
print("ms/step", round(d["ms_per_step"],1), "value", f"{d['value']:.3e}", "gemm TF", round(d["roofline"]["achieved"],1), "solve_ms", round(d["solve_ms"],1), "resid", d["solve_residual"])
print({k: round(v,1) for k,v in d["kernel_ms_per_step"].items()})
PY
