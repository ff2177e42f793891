#!/bin/bash
# Several GPU steps in one gpurun call; each step has its own time limit and the chain stops at the
# first failure.  Usage: tools/gpu_multi.sh TAG "step1 cmd" "step2 cmd" ...
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
i=0
for c in "$@"; do
  i=$((i+1))
  echo "== step $i: $c"
  bash -c "$c" > gpurun_out/${TAG}_step$i.log 2>&1
  rc=$?
  tail -25 gpurun_out/${TAG}_step$i.log
  if [ $rc -ne 0 ]; then echo "step $i failed rc=$rc"; exit $rc; fi
done
