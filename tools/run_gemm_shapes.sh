set -o pipefail
cd sharedmemsparselu.jl_amd
timeout -k 10 100 ./tools/gemm_bench "$@" > ../gpurun_out/gb_s.txt 2>&1
