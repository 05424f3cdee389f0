#!/bin/bash
# GEMV launch-shape re-sweep (graph-timed) over the 70B shapes and their column shards
set -e
export PYTHONPATH=torchao-fork_amd TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u experiments/sweep_gemv.py --graph 10240x8192 8192x8192 57344x8192 8192x28672 1280x8192 1024x8192 7168x8192 1024x28672 3584x8192 2048x8192 > gpurun_out/sweep_gemv_70b_r6r.jsonl
grep BEST gpurun_out/sweep_gemv_70b_r6r.jsonl
