# Round profile on one MI355X (run via gpurun from the repo root): GPU tests, full bench,
# rocprofv3 kernel stats, and the two PMC passes (FETCH_SIZE, WRITE_SIZE) for HBM traffic.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/tgpu.log 2>&1; echo PYTEST $? >> gpurun_out/tgpu.log
timeout -k 10 300 python bench.py > gpurun_out/p_bench.json 2> gpurun_out/p_bench.log || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p_kt -o kt --output-format csv -- python3 bench.py --no-cpu --steps 2 --warmup 1 > gpurun_out/p_kt.json 2> gpurun_out/p_kt.log || exit 1
