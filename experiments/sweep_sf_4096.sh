#!/bin/bash
# int4 M = 128 4096x4096 single-fetch launch shapes (bn, wm, splits, stages, a, ks; loaders
# 1 off / 2 on) timed one process each: GPU-box step, bash experiments/sweep_sf_4096.sh TAG
export PYTHONPATH=torchao-fork_amd TMPDIR=/tmp
O=gpurun_out/$1.jsonl
: > $O
for spec in "64,2,4,4,0,0 0" "32,2,2,3,0,0 1" "32,2,2,4,0,0 1" "32,2,4,4,0,0 1" "32,4,2,4,0,0 1" "32,2,2,4,0,0 2" "32,2,4,4,0,0 2" "64,2,2,4,0,0 2" "64,4,4,4,0,0 2" "64,2,8,4,0,0 2" "128,2,2,4,0,0 1" "128,4,2,3,0,0 1"; do
  set -- $spec
  timeout -k 10 120 python -u experiments/time_sf_cfg.py int4 128x4096x4096 $1 $2 >> $O 2>> ${O%.jsonl}.err || echo "{\"cfg\": \"$1\", \"loaders\": $2, \"failed\": true}" >> $O
done
cat $O
