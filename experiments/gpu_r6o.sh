#!/bin/bash
# GEMV launch-shape re-sweep after the byte-permute decode (graph-timed); wqkv without its seam
set -e
export PYTHONPATH=torchao-fork_amd TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/sweep_gemv_r6o.jsonl
: > $O
timeout -k 10 500 python -u experiments/sweep_gemv.py --graph 4096x4096 6144x4096 14336x4096 4096x14336 28672x4096 >> $O
timeout -k 10 200 python -u experiments/time_partials.py 128x6144x4096 "64,2,2,3,0,0,1;64,2,4,4,0,0,2" 3 > gpurun_out/partials_wqkv_r6o.jsonl
grep BEST $O; cat gpurun_out/partials_wqkv_r6o.jsonl
