# refactor bench: rocBLAS routing (current default) vs hand-written tiles only
set -o pipefail
cd $GRAFT_REPO_ROOT
for V in default norb; do
  if [ $V = norb ]; then export SMLU_NO_ROCBLAS=1; fi
  timeout -k 10 300 python bench.py --no-cpu --no-configs --steps 5 > gpurun_out/r3g_bench_$V.json 2> gpurun_out/r3g_bench_$V.log || { echo BENCH FAIL $V; tail -20 gpurun_out/r3g_bench_$V.log; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r3g_bench_$V.json')); print('$V', round(d['ms_per_step'],1), round(d['roofline']['frac'],3), {k: round(v,1) for k,v in d['kernel_ms_per_step'].items()}, round(d['solve_ms'],2), round(d['solve_8rhs_ms'],1))"
done
