# Dev round trip on one MI355X: GPU tests, then the default bench (no CPU baseline).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tgpu.log 2>&1 || { echo PYTEST FAIL; tail -30 gpurun_out/tgpu.log; exit 1; }
timeout -k 10 200 python bench.py --no-cpu > gpurun_out/b_def.json 2> gpurun_out/b_def.log || exit 1
