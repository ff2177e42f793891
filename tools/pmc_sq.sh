#!/bin/bash
# Dev (via gpurun from the repo root): one PMC pass of LDS bank conflicts and matrix-pipe busy cycles
# over the 128 GEMM tile dispatches of one eager 128^3 factorization.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export SMLU_NO_GRAPH=1
timeout -s KILL 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE \
  --kernel-include-regex "k_gemm128_mfma3" -d gpurun_out/pmcsq_128 -o pmc --output-format csv -- python3 tools/pmc_factor.py 128 \
  > gpurun_out/pmcsq_128.log 2>&1 || { echo PMC FAIL; tail -5 gpurun_out/pmcsq_128.log; exit 1; }
echo PMC OK
