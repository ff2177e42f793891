# Per-launch GEMM efficiency of the 128^3 refactor (via gpurun from the repo root): the schedule
# dump + a rocprofv3 kernel trace of bench.py, paired by tools/gemm_launch_report.py.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export SMLU_DUMP_LAUNCHES=$GRAFT_REPO_ROOT/gpurun_out/launches_128.csv
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/gl_kt -o kt --output-format csv -- python3 bench.py --no-cpu --no-configs --steps 1 --warmup 1 > gpurun_out/gl_kt.json 2> gpurun_out/gl_kt.log || { echo GL KT FAIL; tail gpurun_out/gl_kt.log; exit 1; }
f=$(find gpurun_out/gl_kt -name "kt_kernel_trace.csv" | head -1)
python tools/gemm_launch_report.py gpurun_out/launches_128.csv $f | tee gpurun_out/gemm_launch_report.txt
