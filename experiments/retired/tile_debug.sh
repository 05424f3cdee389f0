#!/bin/bash
# Variant builds of the tile GEMM (csrc/gemm_tile.hip), CPU side: every other object comes from
# the product build (torchao-fork_amd/csrc/build), only gemm_tile.o is rebuilt per variant.
#   bash experiments/tile_debug.sh build   -> experiments/build/libtiledbg{0..5}.so, libtilestamps.so
#   bash experiments/tile_debug.sh run     -> time experiments/ab_tile.py --quick on each (GPU side)
# TAO_TILE_DEBUG: 0 normal, 1 no x loads, 2 no weight loads, 3 no MFMAs, 4 no B-image stores,
# 5 no dequant/conversion. Timing only.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
C="$R/torchao-fork_amd/csrc"
B="$R/experiments/build"
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -munsafe-fp-atomics"
if [ "$1" = build ]; then
  mkdir -p "$B"
  OTHERS=$(ls "$C"/build/*.o | grep -v gemm_tile.o)
  for v in 0 1 2 3 4 5 6 7; do
    /opt/rocm/bin/hipcc $FLAGS -DTAO_TILE_DEBUG=$v -c "$C/gemm_tile.hip" -o "$B/gemm_tile_dbg$v.o"
    /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -Wl,-rpath,/opt/rocm/lib $OTHERS \
      "$B/gemm_tile_dbg$v.o" -o "$B/libtiledbg$v.so"
  done
  /opt/rocm/bin/hipcc $FLAGS -DTAO_TILE_STAMPS=1 -c "$C/gemm_tile.hip" -o "$B/gemm_tile_stamps.o"
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -Wl,-rpath,/opt/rocm/lib $OTHERS \
    "$B/gemm_tile_stamps.o" -o "$B/libtilestamps.so"
else
  for v in 0 1 2 3 4 5 6 7; do
    echo "variant $v"
    TORCHAO_MI355X_LIB="$B/libtiledbg$v.so" timeout -k 10 200 python3 "$R/experiments/ab_tile.py" --quick
  done
fi
