#!/bin/bash
# Build the C-ABI library with each TAO_GEMM_DEBUG variant into experiments/build/ (CPU side),
# or time one configuration on every variant (GPU side): bash experiments/gemm_debug.sh run ARGS
# Variants (gemm_mfma.hip TAO_GEMM_DEBUG): 0 normal, 1 no x loads, 2 no weight loads,
# 3 no x LDS staging (A fragments from registers), 4 no per-step barrier, 5 no global loads at
# all (1 + 2). Timing only.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
if [ "$1" = build ]; then
  for v in 0 1 2 3 4 5; do
    make -s -C "$R/torchao-fork_amd/csrc" -j8 OBJDIR="$R/experiments/build/obj$v" \
      OUT="$R/experiments/build/libdbg$v.so" \
      CXXFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -munsafe-fp-atomics -DTAO_GEMM_DEBUG=$v"
  done
else
  shift
  for v in 0 1 2 3 4 5; do
    echo -n "variant $v: "
    TORCHAO_MI355X_LIB="$R/experiments/build/libdbg$v.so" timeout -k 10 120 python3 "$R/experiments/prof_gemm.py" "$@" | tail -1
  done
fi
