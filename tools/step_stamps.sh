#!/bin/bash
# Build the -DDTSIM_STAMPS diagnostic library (on the CPU host, before gpurun).
cd "$(dirname "$0")/.."
C=aido1_amd/csrc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -shared -std=c++17 -ffp-contract=off \
  -munsafe-fp-atomics -mllvm -pragma-unroll-threshold=1000000 -DDTSIM_STAMPS -o aido1_amd/libdtsim_stamps.so \
  $C/dtsim.hip $C/dtrender.hip $C/dtreplay.hip $C/dtactor.hip $C/dtconv.hip
