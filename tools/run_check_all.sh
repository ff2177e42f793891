# Every -m gpu test (no stop at the first failure), smoke, then the default bench line (via gpurun
# from the repo root): bash tools/run_check_all.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-chk}
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR|SKIPPED" gpurun_out/${T}_tests.log | tail -40
tail -2 gpurun_out/${T}_tests.log
# a test failure (pytest exit 1) lets the next steps run; a timeout, crash or collection error stops here
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "PYTEST EXIT $rc"; exit $rc; fi
[ $rc -eq 1 ] && echo "TESTS FAILED (continuing)"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { echo SMOKE FAIL; tail -20 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
timeout -k 10 400 python bench.py --no-cpu > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.log || { echo BENCH FAIL; tail -20 gpurun_out/${T}_bench.log; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/${T}_bench.json'))
print('ms_per_step', d['ms_per_step'], 'value', d['value'], 'frac', d['roofline']['frac'])
print({k: v for k, v in d.items() if 'solve' in k})
"
exit 0
