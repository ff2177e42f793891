# GEMM tile comparison on the refactor's shapes: t64 (VALU reference), t129 (MFMA v1), t130 (MFMA v2);
# bitwise difference against t64 and TFLOP/s.  Then PMC counters of v1 vs v2 on one big shape.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT/sharedmemsparselu.jl_amd
S="8192,8192,8192 16000,16000,384 16000,16000,1536 12000,12000,3700 9000,9000,2300 3000,3000,256 18000,384,384 1000,1000,300 12000,12000,64 777,1333,129"
GB_TILES=64,129,130 timeout -k 10 200 ./tools/gemm_bench $S > ../gpurun_out/gemm_v2_cmp.txt 2>&1 || { cat ../gpurun_out/gemm_v2_cmp.txt; exit 1; }
cat ../gpurun_out/gemm_v2_cmp.txt
for T in 129 130; do
  GB_TILES=$T timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -d ../gpurun_out/pmc_gemm_t$T -o pmc -- ./tools/gemm_bench 8192,8192,8192 > ../gpurun_out/pmc_gemm_t$T.log 2>&1 || { tail ../gpurun_out/pmc_gemm_t$T.log; exit 1; }
done
echo PMC-DONE
