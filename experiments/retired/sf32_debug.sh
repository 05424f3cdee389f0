#!/bin/bash
# Timing-only variant builds of the 32x32x16 int4 single-fetch kernel (TAO_SF32_DEBUG 1-4, see
# gemm_sf32.hip), each linked into experiments/build/libsf32dbg<N>.so. CPU-side build step.
set -e
cd "$(dirname "$0")/.."
B=experiments/build
mkdir -p $B/sf32dbg
for v in 1 2 3 4; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-function -munsafe-fp-atomics \
    -fno-slp-vectorize -DTAO_SF32_DEBUG=$v -c torchao-fork_amd/csrc/gemm_sf32.hip -o $B/sf32dbg/gemm_sf32_$v.o
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -Wl,-rpath,/opt/rocm/lib -Wl,-z,defs \
    $(ls torchao-fork_amd/csrc/build/*.o | grep -v "/gemm_sf32.o") $B/sf32dbg/gemm_sf32_$v.o -o $B/libsf32dbg$v.so
done
