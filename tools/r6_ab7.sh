#!/bin/bash
# Round-6 dev (via gpurun from the repo root): fused-panel phase trace (build_trace library), then
# A/B of s_setprio(1)/(0) around each MFMA quad of the 128 tile (var/prio.so) vs the committed build.
set -o pipefail
mkdir -p gpurun_out
SMLU_LIB=$PWD/sharedmemsparselu.jl_amd/build_trace/libsmlu_ptrace.so timeout -k 10 300 python tools/panel_trace.py > gpurun_out/panel_trace.txt 2>gpurun_out/panel_trace.log || exit 1
cat gpurun_out/panel_trace.txt
bash tools/ab_libs.sh "var/base3.so var/prio.so var/base3.so var/prio.so" || exit 1
