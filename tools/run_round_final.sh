# End-of-round evidence (via gpurun from the repo root): every -m gpu test, smoke and the bench line
# (tools/run_check_all.sh), the rocprofv3 kernel statistics and PMC passes of the refactor
# (tools/profile_round.sh) and the solve's kernel trace (tools/profile_solve.sh).
#   bash tools/run_round_final.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-final}
bash tools/run_check_all.sh $T || exit 1
bash tools/profile_round.sh 128 > gpurun_out/${T}_profile.txt 2>&1 || { tail -5 gpurun_out/${T}_profile.txt; exit 1; }
tail -2 gpurun_out/${T}_profile.txt
bash tools/profile_solve.sh 128 > gpurun_out/${T}_solve_prof.txt 2>&1 || { tail -5 gpurun_out/${T}_solve_prof.txt; exit 1; }
tail -16 gpurun_out/${T}_solve_prof.txt
