#!/bin/bash
# A/B of the Schur-update GEMM tiles in isolation (sharedmemsparselu.jl_amd/tools/gemm_bench).
# Usage: tools/gemm_ab.sh TAG TILES  (e.g. "130,131")
set -o pipefail
TAG=${1:-ab}; TILES=${2:-130,131}
mkdir -p gpurun_out
cd sharedmemsparselu.jl_amd
GB_TILES=$TILES timeout -k 10 300 ./tools/gemm_bench 8192,8192,8192 16000,16000,384 6000,6000,384 3000,3000,384 12000,12000,6000 16384,16384,2048 4096,16384,384 > ../gpurun_out/${TAG}_gemm.txt 2>&1
rc=$?
cat ../gpurun_out/${TAG}_gemm.txt
exit $rc
