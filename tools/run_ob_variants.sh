# Refactor time for blocking variants (via gpurun from the repo root): bench.py lines without the
# CPU baseline and configs, one per "VAR=value" argument (default: OB 384/512/768, SB 768/1536).
set -o pipefail
cd $GRAFT_REPO_ROOT
for v in ${@:-SMLU_OB=384 SMLU_OB=512 SMLU_OB=768 SMLU_SB=768 SMLU_SB=1536}; do
  tag=$(echo $v | tr '=' '_')
  env $v timeout -k 10 300 python bench.py --no-cpu --no-configs --steps 3 --warmup 1 > gpurun_out/var_$tag.json 2> gpurun_out/var_$tag.log || { echo VAR $v FAIL; tail -5 gpurun_out/var_$tag.log; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/var_$tag.json'))
print('$v', round(d['ms_per_step'],1), 'ms', 'gemm frac', round(d['roofline']['frac'],3), {k: round(v,1) for k, v in (d.get('kernel_ms_per_step') or {}).items()})
"
done
