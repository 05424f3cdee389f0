#!/bin/bash
# Variant builds for A/B timing: each NAME=SRC:DEFINES links csrc/SRC built with DEFINES (in place
# of its shipped object) into experiments/build/libvar_NAME.so. CPU-side step.
#   bash experiments/variant.sh il=gemm_sf:-DTAO_SF_IL=1
set -e
cd "$(dirname "$0")/.."
B=experiments/build
mkdir -p $B/varobj
for pair in "$@"; do
  name=${pair%%=*}; rest=${pair#*=}; src=${rest%%:*}; defs=${rest#*:}
  extra=""
  case $src in gemm_sf|gemm_sf32|attn_mfma) extra=-fno-slp-vectorize;; esac
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-function -munsafe-fp-atomics \
    $extra $defs -c torchao-fork_amd/csrc/$src.hip -o $B/varobj/${src}_$name.o
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -Wl,-rpath,/opt/rocm/lib -Wl,-z,defs \
    $(ls torchao-fork_amd/csrc/build/*.o | grep -v "/$src.o") $B/varobj/${src}_$name.o -o $B/libvar_$name.so
done
