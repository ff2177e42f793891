set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/run_check_all.sh r4f && timeout -k 10 200 python tools/solve_bench.py 128 > gpurun_out/solve_pf.json 2> gpurun_out/solve_pf.log && cat gpurun_out/solve_pf.json && bash tools/profile_solve.sh 128 > gpurun_out/sol_prof_pf.txt 2>&1 && tail -16 gpurun_out/sol_prof_pf.txt && bash tools/run_ob_variants.sh SMLU_OB=512 SMLU_SB=768
