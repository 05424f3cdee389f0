#!/bin/bash
# GPU-box step: experiments/gemv_graph_time.py over a few tao_tune_int4_gemv launch shapes
# (rpw,wk,g,occ; "" = built-in) for the shapes in SHAPES. bash experiments/gemv_shape_sweep.sh TAG
cd "$(dirname "$0")/.." || exit 1
export PYTHONPATH=torchao-fork_amd TMPDIR=/tmp
O=gpurun_out/$1.jsonl
: > $O
for t in "" 4,1,4,0 2,1,4,0 4,2,1,0 4,1,2,0 2,2,1,0 8,1,2,0 4,1,4,8; do
  TUNE=$t timeout -k 10 120 python -u experiments/gemv_graph_time.py >> $O 2>> gpurun_out/$1.err || exit $?
done
cat $O
