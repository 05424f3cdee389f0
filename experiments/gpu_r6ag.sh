#!/bin/bash
# no per-step barrier in the 16x16 loader kernel (timing only: races) (variant lib)
set -e
export PYTHONPATH=torchao-fork_amd TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/ab_sf_nobar_r6ag.jsonl
: > $O
for i in 1 2; do
  timeout -k 10 200 python -u experiments/time_routes.py >> $O
  TORCHAO_MI355X_LIB=experiments/ablib/libsf_nobar.so timeout -k 10 200 python -u experiments/time_routes.py >> $O
done
grep int4 $O
