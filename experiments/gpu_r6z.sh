#!/bin/bash
# interleaved A/B of decode-fused launch shapes with waves along K (70B and 8B)
set -e
export PYTHONPATH=torchao-fork_amd TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/ab_decode_shape_r6z.jsonl
: > $O
timeout -k 10 300 python -u experiments/ab_decode_shape.py 70b wqkv_rope "0,0,0,0;4,2,1,8;4,2,1,4;4,2,2,4;2,2,1,4;2,2,2,4" 5 >> $O
timeout -k 10 300 python -u experiments/ab_decode_shape.py 70b w13_swiglu "0,0,0,0;4,2,1,4;4,2,2,4" 5 >> $O
timeout -k 10 300 python -u experiments/ab_decode_shape.py 8b wqkv_rope "0,0,0,0;2,2,1,4;2,2,2,4;4,2,1,8" 5 >> $O
timeout -k 10 300 python -u experiments/ab_decode_shape.py 8b w13_swiglu "0,0,0,0;4,2,1,4;4,2,2,4" 5 >> $O
cat $O
