#!/bin/bash
# Ring-depth variants of the MFMA skinny GEMM (gemm_mfma.hip TAO_GEMM_DEPTH): build on the CPU
# side (bash experiments/gemm_depth.sh build), time on the GPU side
# (bash experiments/gemm_depth.sh run PATH M N K BM KG SPLITS).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
DEPTHS="2 3 4 6 8"
if [ "$1" = build ]; then
  for d in $DEPTHS; do
    make -s -C "$R/torchao-fork_amd/csrc" -j8 OBJDIR="$R/experiments/build/depth$d" \
      OUT="$R/experiments/build/libdepth$d.so" \
      CXXFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -munsafe-fp-atomics -DTAO_GEMM_DEPTH=$d"
  done
else
  shift
  for d in $DEPTHS; do
    echo -n "depth $d: "
    TORCHAO_MI355X_LIB="$R/experiments/build/libdepth$d.so" timeout -k 10 120 python3 "$R/experiments/prof_gemm.py" "$@" | tail -1
  done
fi
