#!/bin/bash
# the new K = 8192 launch shapes on the unmeasured 2- / 4-way shard shapes: built-in (0,0,0,0) vs candidates
set -e
export PYTHONPATH=torchao-fork_amd TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/ab_gemv_shards_r6t.jsonl
: > $O
timeout -k 10 200 python -u experiments/ab_gemv_shape.py 5120x8192 "0,0,0,0;4,4,1,4;4,2,2,4;4,1,2,4" 3 >> $O
timeout -k 10 200 python -u experiments/ab_gemv_shape.py 28672x8192 "0,0,0,0;4,4,1,4;4,2,2,4;4,1,4,4" 3 >> $O
timeout -k 10 200 python -u experiments/ab_gemv_shape.py 14336x8192 "0,0,0,0;4,4,1,4;4,1,1,4;4,1,2,4" 3 >> $O
timeout -k 10 200 python -u experiments/ab_gemv_shape.py 2560x8192 "0,0,0,0;2,4,1,0;4,2,1,4" 3 >> $O
timeout -k 10 200 python -u experiments/ab_gemv_shape.py 4096x8192 "0,0,0,0;4,1,1,4;2,4,1,0" 3 >> $O
cat $O
