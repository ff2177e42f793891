# dev: kernel trace of the bench (2 steps) for per-launch analysis.  bash tools/run_r3o.sh TAG [env...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=$1; shift
rm -rf gpurun_out/$T
env "$@" timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/$T -o kt --output-format csv -- python3 bench.py --no-cpu --no-configs --steps 2 --warmup 1 > gpurun_out/$T.json 2> gpurun_out/$T.log || { tail gpurun_out/$T.log; exit 1; }
echo TRACE OK
