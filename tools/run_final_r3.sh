# Final round-3 check of the frozen source (via gpurun from the repo root): every -m gpu test,
# smoke, the default bench line, then the rocprofv3 kernel trace + PMC passes (tools/profile_r3.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/run_round_check.sh fin && bash tools/profile_r3.sh 128
