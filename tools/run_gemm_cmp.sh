set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
S="12000,12000,64 12000,12000,256 12000,12000,1024 20000,5000,256 4096,4096,4096 3000,3000,256 1000,1000,300 18000,192,64"
cd sharedmemsparselu.jl_amd
timeout -k 10 100 ./tools/gemm_bench $S > ../gpurun_out/gb_p.txt 2>&1 || exit 1

cd ..
timeout -k 10 200 python bench.py --no-cpu > gpurun_out/b_def.json 2> gpurun_out/b_def.log || exit 1
