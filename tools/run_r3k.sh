# look-ahead variants (dev): default vs SMLU_LOOKAHEAD=1 with/without graph and CU reserve
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run() { echo "== $1"; env $2 timeout -k 10 200 python bench.py --no-cpu --no-configs --steps 3 > gpurun_out/r3k_$1.json 2> gpurun_out/r3k_$1.log || { tail -5 gpurun_out/r3k_$1.log; return 1; }; python3 -c "import json; d=json.load(open('gpurun_out/r3k_$1.json')); print(d['ms_per_step'], d['solve_ms'], {k: round(v,1) for k,v in d['kernel_ms_per_step'].items()})"; }
run base "SMLU_X=0" && run la "SMLU_LOOKAHEAD=1" && run la_nog "SMLU_LOOKAHEAD=1 SMLU_NO_GRAPH=1" && run la_res "SMLU_LOOKAHEAD=1 SMLU_SIDE_RESERVE=2" && run la_res_nog "SMLU_LOOKAHEAD=1 SMLU_SIDE_RESERVE=2 SMLU_NO_GRAPH=1"
