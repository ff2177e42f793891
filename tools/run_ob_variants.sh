# Refactor time for outer-block widths (via gpurun from the repo root): bench.py lines without the
# CPU baseline and configs, one per SMLU_OB value.
set -o pipefail
cd $GRAFT_REPO_ROOT
for ob in ${@:-384 512 768}; do
  SMLU_OB=$ob timeout -k 10 300 python bench.py --no-cpu --no-configs --steps 3 --warmup 1 > gpurun_out/ob_$ob.json 2> gpurun_out/ob_$ob.log || { echo OB $ob FAIL; tail -5 gpurun_out/ob_$ob.log; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/ob_$ob.json'))
print('OB $ob', round(d['ms_per_step'],1), 'ms', 'gemm frac', round(d['roofline']['frac'],3), 'kinds', {k: round(v,1) for k, v in (d.get('kernel_ms_per_step') or {}).items()})
"
done
