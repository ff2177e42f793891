# Dev round trip: GPU tests, then bench variants given as env strings (first = default env).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tgpu.log 2>&1 || { echo PYTEST FAIL; tail -30 gpurun_out/tgpu.log; exit 1; }
i=0
for v in "$@"; do
  i=$((i+1))
  env $v timeout -k 10 200 python bench.py --no-cpu > gpurun_out/var_$i.json 2> gpurun_out/var_$i.log || exit 1
done
