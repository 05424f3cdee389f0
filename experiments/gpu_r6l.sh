#!/bin/bash
# wo / w2 partials form under launch-shape overrides (experiments/time_partials.py)
set -e
export PYTHONPATH=torchao-fork_amd TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/partials_r6l.jsonl
: > $O
timeout -k 10 240 python -u experiments/time_partials.py 128x4096x14336 "64,2,4,4,0,0,2;64,2,8,4,0,0,2;64,2,8,3,0,0,2;128,2,8,3,0,0,1;128,2,8,2,0,0,1;128,4,8,3,0,0,1;128,2,4,3,0,0,1;256,2,16,2,0,0,1;256,2,8,2,0,0,1;64,2,7,4,0,0,2" >> $O
timeout -k 10 240 python -u experiments/time_partials.py 128x4096x4096 "64,2,4,4,0,0,2;64,2,8,4,0,0,2;128,2,8,3,0,0,1;128,2,8,2,0,0,1;128,4,8,3,0,0,1;256,2,16,2,0,0,1;128,2,4,3,0,0,1" >> $O
cat $O
