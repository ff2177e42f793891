#!/bin/bash
# Round-6 A/B 17 (via gpurun from the repo root): static s_setprio 1 for the odd workgroups of the
# 128 tile (var/sprio.so) vs the committed build (var/base7.so); the 128^3 bench.
set -o pipefail
mkdir -p gpurun_out
bash tools/ab_libs.sh "var/base7.so var/sprio.so var/base7.so var/sprio.so" || exit 1
