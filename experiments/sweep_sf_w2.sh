#!/bin/bash
# int4 M = 128 4096x14336 (w2) and 6144x4096 (wqkv) single-fetch launch shapes (bn, wm, splits,
# stages, a, ks; loaders 1 off / 2 on), one process each. GPU-box step:
#   bash experiments/sweep_sf_w2.sh TAG
export PYTHONPATH=torchao-fork_amd TMPDIR=/tmp
O=gpurun_out/$1.jsonl
: > $O
for spec in "128x4096x14336 64,2,4,4,0,0 0" "128x4096x14336 64,2,8,4,0,0 2" "128x4096x14336 64,4,4,4,0,0 2" "128x4096x14336 64,2,4,3,0,0 2" "128x4096x14336 64,4,8,4,0,0 2" "128x4096x14336 64,2,2,4,0,0 2" "128x4096x14336 64,2,7,4,0,0 2" "128x6144x4096 64,2,2,3,0,0 0" "128x6144x4096 64,2,4,4,0,0 2" "128x6144x4096 64,4,2,4,0,0 2" "128x6144x4096 64,2,3,4,0,0 2"; do
  set -- $spec
  timeout -k 10 120 python -u experiments/time_sf_cfg.py int4 $1 $2 $3 >> $O 2>> ${O%.jsonl}.err || echo "{\"shape\": \"$1\", \"cfg\": \"$2\", \"loaders\": $3, \"failed\": true}" >> $O
done
cat $O
