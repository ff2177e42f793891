# dev: PMC counters of the fused panel kernel (one eager factorization, k_panel_blk dispatches)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export SMLU_NO_GRAPH=1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU --kernel-include-regex "k_panel_blk" -d gpurun_out/pmcP -o p --output-format csv -- python3 tools/pmc_factor.py 128 > gpurun_out/pmcP.log 2>&1 || { tail gpurun_out/pmcP.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_WAVES --kernel-include-regex "k_panel_blk" -d gpurun_out/pmcP2 -o p --output-format csv -- python3 tools/pmc_factor.py 128 > gpurun_out/pmcP2.log 2>&1 || { tail gpurun_out/pmcP2.log; exit 1; }
echo PMC OK
