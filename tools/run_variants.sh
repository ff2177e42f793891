# Bench variants via env (dev): bash tools/run_variants.sh "ENV1=.. ENV2=.." "ENV=.." ...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
i=0
for v in "$@"; do
  i=$((i+1))
  env $v timeout -k 10 200 python bench.py --no-cpu > gpurun_out/var_$i.json 2> gpurun_out/var_$i.log || exit 1
done
