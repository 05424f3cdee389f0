#!/bin/bash
# Variant builds of the 32x32x16 int4 single-fetch kernel for A/B timing: each NAME=DEFINES pair
# links gemm_sf32.hip built with DEFINES into experiments/build/libsf32<NAME>.so. CPU-side step.
#   bash experiments/sf32_variant.sh il=-DTAO_SF32_IL=1
set -e
cd "$(dirname "$0")/.."
B=experiments/build
mkdir -p $B/sf32var
for pair in "$@"; do
  name=${pair%%=*}; defs=${pair#*=}
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-function -munsafe-fp-atomics \
    -fno-slp-vectorize $defs -c torchao-fork_amd/csrc/gemm_sf32.hip -o $B/sf32var/gemm_sf32_$name.o
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -Wl,-rpath,/opt/rocm/lib -Wl,-z,defs \
    $(ls torchao-fork_amd/csrc/build/*.o | grep -v "/gemm_sf32.o") $B/sf32var/gemm_sf32_$name.o -o $B/libsf32$name.so
done
