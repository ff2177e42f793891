# Round profile (via gpurun from the repo root): rocprofv3 kernel stats of the bench, then the
# PMC passes (FETCH_SIZE, WRITE_SIZE, one counter per pass) over the k_gemm* dispatches and over
# every kernel of one eager factorization.  bash tools/profile_round.sh N
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
N=${1:-128}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p_kt -o kt --output-format csv -- python3 bench.py --no-cpu --no-configs --steps 2 --warmup 1 > gpurun_out/p_kt.json 2> gpurun_out/p_kt.log || { echo KT FAIL; tail gpurun_out/p_kt.log; exit 1; }
export SMLU_NO_GRAPH=1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-include-regex "k_gemm|Cijk" -d gpurun_out/pmc_${c}_$N -o pmc \
    --output-format csv -- python3 tools/pmc_factor.py $N > gpurun_out/pmc_${c}_$N.log 2>&1 || { echo PMC FAIL $c; tail gpurun_out/pmc_${c}_$N.log; exit 1; }
done
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c -d gpurun_out/pmcall_${c}_$N -o pmc \
    --output-format csv -- python3 tools/pmc_factor.py $N > gpurun_out/pmcall_${c}_$N.log 2>&1 || { echo PMCALL FAIL $c; tail gpurun_out/pmcall_${c}_$N.log; exit 1; }
done
echo PROFILE OK
