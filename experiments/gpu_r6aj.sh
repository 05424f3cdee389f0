#!/bin/bash
# prologue depth: the 4096-column route shape at K = 1024 / 4096 with 2 / 3 / 4 stages (loaders on)
set -e
export PYTHONPATH=torchao-fork_amd TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/sf_stages_r6aj.jsonl
: > $O
for i in 1 2; do
for K in 1024 4096; do
for NS in 2 3 4; do
  timeout -k 10 120 python -u experiments/time_sf_cfg.py int4 128x4096x$K 64,2,4,$NS,0,0 2 >> $O
done
done
done
cat $O
