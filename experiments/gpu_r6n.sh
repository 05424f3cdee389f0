#!/bin/bash
# w2 / wo partials: route vs 128-column S 8, interleaved passes in one process
set -e
export PYTHONPATH=torchao-fork_amd TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/partials_r6n.jsonl
: > $O
timeout -k 10 300 python -u experiments/time_partials.py 128x4096x14336 "128,2,8,2,0,0,1;128,2,8,3,0,0,1;64,2,4,3,0,0,2" 6 >> $O
timeout -k 10 300 python -u experiments/time_partials.py 128x4096x4096 "128,2,8,2,0,0,1;64,2,4,3,0,0,2" 6 >> $O
cat $O
