# rocprofv3 kernel trace + stats of a short bench run (dev): bash tools/run_ktrace.sh TAG
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-kt}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$T -o kt --output-format csv -- python3 bench.py --no-cpu --steps 1 --warmup 1 > gpurun_out/$T.json 2> gpurun_out/$T.log
