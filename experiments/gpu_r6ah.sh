#!/bin/bash
# fixed vs per-step cost of the 16x16 int4 kernel: the 4096^2 route's launch shape at K = 1024..16384
set -e
export PYTHONPATH=torchao-fork_amd TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/sf_ksweep_r6ah.jsonl
: > $O
for i in 1 2; do
for K in 1024 2048 4096 8192 16384; do
  timeout -k 10 120 python -u experiments/time_sf_cfg.py int4 128x4096x$K 64,2,4,4,0,0 2 >> $O
  timeout -k 10 120 python -u experiments/time_sf_cfg.py int4 128x4096x$K 64,2,1,4,0,0 2 >> $O
done
done
cat $O
