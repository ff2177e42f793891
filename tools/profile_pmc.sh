# HBM traffic of the GEMM kernels (the dominant kernel) from rocprofv3 PMC: FETCH_SIZE and
# WRITE_SIZE in separate passes, counters collected on the k_gemm* dispatches of one eager
# factorization (tools/pmc_factor.py).  Run via gpurun from the repo root: bash tools/profile_pmc.sh N
set -o pipefail
N=${1:-128}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export SMLU_NO_GRAPH=1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 500 rocprofv3 --pmc $c --kernel-include-regex "k_gemm|Cijk" -d gpurun_out/pmc_${c}_$N -o pmc \
    --output-format csv -- python3 tools/pmc_factor.py $N > gpurun_out/pmc_${c}_$N.log 2>&1 || exit 1
done
