# PMC counters of the v2 MFMA tile (gemm_bench, tile 130) on 8192^3 and on the trailing-update
# shape (k = 384), two passes of 8 SQ counters each.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT/sharedmemsparselu.jl_amd
export GB_TILES=130
for S in 8192,8192,8192 16000,16000,384; do
  t=$(echo $S | tr , x)
  timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -d ../gpurun_out/pmcA_$t -o p --output-format csv -- ./tools/gemm_bench $S > ../gpurun_out/pmcA_$t.log 2>&1 || { tail ../gpurun_out/pmcA_$t.log; exit 1; }
  timeout -s KILL 60 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_SCA -d ../gpurun_out/pmcB_$t -o p --output-format csv -- ./tools/gemm_bench $S > ../gpurun_out/pmcB_$t.log 2>&1 || { tail ../gpurun_out/pmcB_$t.log; exit 1; }
done
echo PMC-DONE
