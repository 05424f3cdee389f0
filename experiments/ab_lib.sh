#!/bin/bash
# Same-box A/B of two builds of the C-ABI library on the prefill MFMA GEMMs (auto shape):
# bash experiments/ab_lib.sh LIB_B [reps]; A = the in-tree library. Alternates A, B, A, B.
set -e
B=$1
for cfg in "int4 128 4096 4096" "int4 128 28672 4096" "int8wo 128 4096 4096" "int4 32 4096 4096" "int8dyn 128 4096 4096"; do
  for rep in 1 2; do
    echo -n "A "; timeout -k 10 60 python3 experiments/prof_gemm.py $cfg 0 0 0 40
    echo -n "B "; TORCHAO_MI355X_LIB=$B timeout -k 10 60 python3 experiments/prof_gemm.py $cfg 0 0 0 40
  done
done
