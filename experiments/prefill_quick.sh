#!/bin/bash
# Kernel µs of the prefill MFMA GEMMs (auto launch shape), XCD-grouped (order 0) and plain
# (order 1) workgroup order, one line per config. usage: bash THIS [orders]
set -e
ORDERS=${1:-"0 1"}
for cfg in "int8dyn 128 4096 4096" "int8dyn 128 28672 4096" "int8dyn 128 14336 4096" "int4 128 4096 4096" "int4 128 28672 4096" "int4 128 6144 4096" "int8wo 128 4096 4096" "int4 512 4096 4096" "int4 32 4096 4096"; do
  for o in $ORDERS; do
    timeout -k 10 60 python3 experiments/prof_gemm.py $cfg 0 0 0 40 $o
  done
done
