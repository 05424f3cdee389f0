#!/bin/bash
# w2 partials shapes (more), w1||w3 on 256-column tiles of the 32x32x16 kernel
set -e
export PYTHONPATH=torchao-fork_amd TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/partials_r6m.jsonl
: > $O
timeout -k 10 240 python -u experiments/time_partials.py 128x4096x14336 "128,2,8,2,0,0,1;128,2,8,4,0,0,1;128,2,7,2,0,0,1;128,2,16,2,0,0,1;128,2,14,2,0,0,1;128,2,8,2,0,0,2;128,2,4,2,0,0,1;128,2,16,3,0,0,1" >> $O
P=gpurun_out/w13_r6m.jsonl
: > $P
for spec in "128,1,1,3,0,0 0" "256,1,2,3,0,0 1" "256,1,2,2,0,0 1" "256,1,1,3,0,0 1" "256,1,2,3,0,2 1" "128,1,2,3,0,0 2" "128,1,2,3,0,0 1" "256,1,2,3,0,0 2"; do
  set -- $spec
  timeout -k 10 120 python -u experiments/time_sf_cfg.py int4 128x28672x4096 $1 $2 >> $P 2>> ${P%.jsonl}.err || echo "{\"cfg\": \"$1\", \"loaders\": $2, \"failed\": true}" >> $P
done
cat $O $P
