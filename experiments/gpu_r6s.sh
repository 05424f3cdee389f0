#!/bin/bash
# interleaved A/B of the 70B-shape GEMV launch shapes the r6r sweep prefers
set -e
export PYTHONPATH=torchao-fork_amd TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/ab_gemv_70b_r6s.jsonl
: > $O
timeout -k 10 200 python -u experiments/ab_gemv_shape.py 8192x8192 "4,4,1,4;4,1,1,4;4,2,1,4" 5 >> $O
timeout -k 10 200 python -u experiments/ab_gemv_shape.py 10240x8192 "4,4,1,4;4,1,1,4;4,2,2,4" 5 >> $O
timeout -k 10 300 python -u experiments/ab_gemv_shape.py 57344x8192 "8,4,1,4;8,2,1,4;4,1,1,4" 5 >> $O
timeout -k 10 200 python -u experiments/ab_gemv_shape.py 7168x8192 "4,4,1,4;4,1,1,4" 5 >> $O
timeout -k 10 200 python -u experiments/ab_gemv_shape.py 1024x8192 "2,2,1,0;2,4,1,0" 5 >> $O
timeout -k 10 200 python -u experiments/ab_gemv_shape.py 1280x8192 "2,2,1,0;2,4,1,0" 5 >> $O
cat $O
