#!/bin/bash
# no dequantisation in the 16x16 kernel (raw nibble dwords as the B fragment) (variant lib)
set -e
export PYTHONPATH=torchao-fork_amd TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/ab_sf_nodeq_r6ae.jsonl
: > $O
for i in 1 2; do
  timeout -k 10 200 python -u experiments/time_routes.py >> $O
  TORCHAO_MI355X_LIB=experiments/ablib/libsf_nodeq.so timeout -k 10 200 python -u experiments/time_routes.py >> $O
done
grep int4 $O
