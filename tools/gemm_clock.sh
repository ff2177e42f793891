#!/bin/bash
# Builds the clock-probe variant of the library (kernels_gemm.hip with -DSMLU_CLOCK_PROBE, every other
# object from the regular build) into sharedmemsparselu.jl_amd/build_clock/; run on the CPU box, then
#   gpurun -- 'SMLU_LIB=$PWD/sharedmemsparselu.jl_amd/build_clock/libsmlu_clock.so python tools/gemm_clock.py'
set -e
cd "$(dirname "$0")/../sharedmemsparselu.jl_amd"
make -s -j8 libsmlu.so
mkdir -p build_clock
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall -Wno-unused-result --offload-arch=gfx950 -munsafe-fp-atomics \
  -DSMLU_CLOCK_PROBE -c csrc/kernels_gemm.hip -o build_clock/kernels_gemm.o
/opt/rocm/bin/hipcc -shared -fPIC -Wl,-z,defs --offload-arch=gfx950 -o build_clock/libsmlu_clock.so \
  $(ls build/*.o | grep -v -e kernels_gemm -e _bench) build_clock/kernels_gemm.o
