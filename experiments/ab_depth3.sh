#!/bin/bash
# Ring depth A/B of the MFMA GEMM: in-tree (2 at BM >= 64) vs TAO_GEMM_DEPTH=3 / 4 builds, on
# the int4 / int8 shapes whose table or heuristic shape has BM 64. Alternates the three builds.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
for cfg in "int4 128 4096 4096" "int4 128 6144 4096" "int4 256 4096 4096" "int4 512 4096 4096" "int4 64 6144 4096" "int8wo 128 4096 4096" "int4 128 4096 14336"; do
  for rep in 1 2; do
    echo -n "D2 "; timeout -k 10 60 python3 $R/experiments/prof_gemm.py $cfg 0 0 0 40
    echo -n "D3 "; TORCHAO_MI355X_LIB=$R/experiments/build/libdepth3.so timeout -k 10 60 python3 $R/experiments/prof_gemm.py $cfg 0 0 0 40
    echo -n "D4 "; TORCHAO_MI355X_LIB=$R/experiments/build/libdepth4.so timeout -k 10 60 python3 $R/experiments/prof_gemm.py $cfg 0 0 0 40
  done
done
