# Dev: PMC counters of the MFMA GEMM tile on one large shape (gemm_bench, tile 129), one pass
# per counter group, plus the shader clock sampled while a long run executes.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B=sharedmemsparselu.jl_amd/tools/gemm_bench
export GB_TILES=${GB_TILES:-129}
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/pmcg1 -o p --output-format csv -- $B 8192,8192,8192 > gpurun_out/pmcg1.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAVES -d gpurun_out/pmcg2 -o p --output-format csv -- $B 8192,8192,8192 > gpurun_out/pmcg2.log 2>&1 || exit 1
( for i in $(seq 1 12); do rocm-smi --showclocks 2>/dev/null | grep -i "sclk" ; sleep 0.5; done ) > gpurun_out/clk.txt &
timeout -k 10 60 $B 16000,16000,8192 16000,16000,8192 > gpurun_out/pmcg_long.txt 2>&1
wait
