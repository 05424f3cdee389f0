#!/bin/bash
# Build the C-ABI library with each TAO_GEMV_DEBUG variant into experiments/build/ (CPU side),
# or time the Llama-3-8B GEMV shapes on every variant (GPU side): bash experiments/gemv_debug.sh run
# Variants (int4_gemv.hip TAO_GEMV_DEBUG): 0 normal, 1 no x loads, 2 no dequant/dot arithmetic,
# 3 no (scale, zero) loads, 4 no cross-lane / cross-wave reduction, 5 = 2 + 4, 6 = weight loads
# only. Timing only.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
if [ "$1" = build ]; then
  for v in 0 1 2 3 4 5 6; do
    make -s -C "$R/torchao-fork_amd/csrc" -j8 OBJDIR="$R/experiments/build/gobj$v" \
      OUT="$R/experiments/build/libgdbg$v.so" \
      CXXFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -munsafe-fp-atomics -DTAO_GEMV_DEBUG=$v"
  done
else
  shift
  for v in 0 1 2 3 4 5 6; do
    echo "variant $v"
    TORCHAO_MI355X_LIB="$R/experiments/build/libgdbg$v.so" timeout -k 10 120 python3 "$R/experiments/probe_graph_shapes.py" "$@"
  done
fi
