#!/bin/bash
# GEMV variant libraries against the shipped one, per-launch graph us (LIBS, SHAPES, OUT override):
# by default the end-of-kernel store: shipped vs no store (timing only) vs sc1 stores
set -e
export PYTHONPATH=torchao-fork_amd TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/${OUT:-ab_gemv_store_r6am}.jsonl
: > $O
for i in 1 2; do
for lib in ${LIBS:-shipped experiments/ablib/libgemv_nostore.so experiments/ablib/libgemv_sc1store.so}; do
  for shape in ${SHAPES:-4096x4096 28672x4096 4096x14336}; do
    if [ $lib = shipped ]; then
      timeout -k 10 120 python -u experiments/ab_gemv_shape.py $shape "0,0,0,0" 3 | sed "s#^{#{\"lib\": \"$lib\", #" >> $O
    else
      TORCHAO_MI355X_LIB=$lib timeout -k 10 120 python -u experiments/ab_gemv_shape.py $shape "0,0,0,0" 3 | sed "s#^{#{\"lib\": \"$lib\", #" >> $O
    fi
  done
done
done
cat $O
