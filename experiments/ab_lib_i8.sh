#!/bin/bash
# Same-box A/B of two library builds on the int8 GEMM shapes (both kernels), alternating A, B.
# bash experiments/ab_lib_i8.sh LIB_B ; A = the in-tree library.
set -e
B=$1
for cfg in "int8dyn 128 4096 4096" "int8dyn 256 4096 4096" "int8dyn 128 28672 4096" "int8dyn 512 14336 4096" "int8wo 128 28672 4096" "int8wo 64 4096 4096"; do
  for rep in 1 2; do
    echo -n "A "; timeout -k 10 60 python3 experiments/prof_gemm.py $cfg 0 0 0 40
    echo -n "B "; TORCHAO_MI355X_LIB=$B timeout -k 10 60 python3 experiments/prof_gemm.py $cfg 0 0 0 40
  done
done
