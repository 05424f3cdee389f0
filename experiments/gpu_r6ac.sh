#!/bin/bash
# interleaved fragment reads in the 16x16 single-fetch kernel (variant lib) vs shipped, A B A B
set -e
export PYTHONPATH=torchao-fork_amd TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/ab_sf_ilr_r6ac.jsonl
: > $O
for i in 1 2; do
  timeout -k 10 200 python -u experiments/time_routes.py >> $O
  TORCHAO_MI355X_LIB=experiments/ablib/libsf_ilr.so timeout -k 10 200 python -u experiments/time_routes.py >> $O
done
cat $O
