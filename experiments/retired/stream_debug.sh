#!/bin/bash
# Build the C-ABI library with each TAO_STREAM_DEBUG variant into experiments/build/ (CPU side),
# or time the stream GEMM on every variant (GPU side): bash experiments/stream_debug.sh run
# Variants (gemm_stream.hip): 0 normal, 1 no fragment reads / MFMAs, 2 no weight DMA,
# 3 no x DMA, 4 no DMA at all. Timing only.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
VARS="0 1 2 3 4"
if [ "$1" = build ]; then
  for v in $VARS; do
    make -s -C "$R/torchao-fork_amd/csrc" -j8 OBJDIR="$R/experiments/build/sobj$v" \
      OUT="$R/experiments/build/libsdbg$v.so" \
      CXXFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -munsafe-fp-atomics -DTAO_STREAM_DEBUG=$v"
  done
else
  for v in $VARS; do
    TORCHAO_MI355X_LIB="$R/experiments/build/libsdbg$v.so" timeout -k 10 120 \
      python3 "$R/experiments/prof_stream.py" --variant $v
  done
fi
